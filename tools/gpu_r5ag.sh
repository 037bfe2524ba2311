set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for L in old new old new; do
  for W in 1 4; do
    echo "== $L $W windows"; VLOG_AMD_LIB=$PWD/abtmp/$L.so timeout -k 10 300 python3 bench.py --windows $W --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-variable 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; print(d['value'], d['config']['token_crc32'], 'comb', k['cross_comb']['ms'])" || exit 1
  done
  echo "== $L variable"; VLOG_AMD_LIB=$PWD/abtmp/$L.so timeout -k 10 300 python3 bench.py --workload variable --steps 3 --warmup 1 --no-cpu-baseline --no-parity 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; c=d['config']; print(d['value'], c['token_crc32'], 'comb', k['cross_comb']['ms'])" || exit 1
done 2>&1 | tee gpurun_out/ab_xcomb_kb.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xattn.py tests/test_gpu_split.py 2>&1 | tail -2
