# rocprofv3 kernel-trace stats of one bench step (env passed through, e.g. VLOG_AMD_XSPLITS=1); TAG names the output
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
TAG=${TAG:-prof}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
F=$(ls $R/gpurun_out/prof_$TAG/*kernel_stats.csv | head -1)
python3 - "$F" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:22]:
    print(f"{float(r['TotalDurationNs'])/3e6:9.1f} ms/step {int(r['Calls'])//3:7d} calls/step {float(r['AverageNs'])/1e3:9.2f} us  {r['Name'][:90]}")
PY
