# smoke() as the driver runs it, then the worker's exact call (sequential and VLOG_AMD_THROUGHPUT) at T=0.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r02.log 2>&1; rc=$?; tail -2 gpurun_out/smoke_r02.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/bench_worker_call.py --temperature 0 --minutes-seq 2 --minutes-tp 30 > gpurun_out/worker_r02_h_t0.json 2> gpurun_out/worker_r02_h_t0.err || { tail -20 gpurun_out/worker_r02_h_t0.err; exit 1; }
cat gpurun_out/worker_r02_h_t0.json
