# One gpurun call, several bench.py lines: BENCHES is a ';'-separated list of "tag|env assignments|bench args" (the
# middle field may be empty).  Every run under its own time limit; the call stops at the first failure (no GPU
# step after a fault).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
IFS=';' read -ra LIST <<< "$BENCHES"
for item in "${LIST[@]}"; do
  tag=${item%%|*}; rest=${item#*|}; envs=${rest%%|*}; args=${rest#*|}
  echo "== $tag: $envs bench.py $args" | tee -a gpurun_out/bench_list.log
  env $envs timeout -k 10 ${BENCH_LIMIT:-300} python3 bench.py $args > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; tail -20 gpurun_out/bench_$tag.err; exit $rc; fi
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$tag.json')); c=d['config']; k=d.get('kernels_one_step',{}); print('$tag', d['value'], d['ms_per_step'], c.get('mean_tokens_per_window'), c.get('decoder_steps'), c.get('active_row_fraction'), d.get('stages_s_per_step'), 'dec_gemm', (k.get('dec_gemm') or {}).get('ms'), 'xattn_us', d.get('roofline',{}).get('avg_launch_us'), 'parity', (d.get('parity') or {}).get('identical'))" | tee -a gpurun_out/bench_list.log
done
