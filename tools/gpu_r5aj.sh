set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xattn.py tests/test_gpu_split.py "tests/test_gpu_logprobs.py::test_config2_base_32_windows_every_step" 2>&1 | tail -2 || exit 1
for L in old new old new; do
  echo "== $L"; VLOG_AMD_LIB=$PWD/abtmp/$L.so timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-parity --no-variable 2>&1 | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_one_step']; print(d['value'], d['config']['token_crc32'], 'comb', k['cross_comb']['ms'], 'decode', d['stages_s_per_step']['decode'])" || exit 1
done 2>&1 | tee gpurun_out/ab_xcomb_prefetch.txt
