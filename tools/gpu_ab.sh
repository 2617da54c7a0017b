# A/B of the Shift_tcn fusion modes on the NTU bench (gpurun -- bash tools/gpu_ab.sh)
#   CASES="mode:minC ..." (default "1:0 0:0 1:128")
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out/ab
for c in ${CASES:-1:0 0:0 1:128}; do
  m=${c%%:*}; k=${c##*:}
  SGCN_TSHIFT_FUSION_MIN_C=$k timeout -k 10 300 python -u bench.py --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/ab/bench_m${m}_k${k}.log 2>&1
  echo "mode $m minC $k: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/bench_m${m}_k${k}.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['step_breakdown_ms'])")"
done
