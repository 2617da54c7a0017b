# A/B of the Shift_tcn fusion modes on the NTU bench (gpurun -- bash tools/gpu_ab.sh)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out/ab
for m in ${MODES:-1 0 2}; do
  SGCN_TSHIFT_FUSION=$m timeout -k 10 300 python -u bench.py --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/ab/bench_m$m.log 2>&1
  echo "mode $m: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/bench_m$m.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['step_breakdown_ms'])")"
done
