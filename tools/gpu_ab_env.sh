# Same-box A/B of environment settings on the NTU bench:
#   gpurun -- 'CASES="SGCN_ASYNC_DW=0 SGCN_ASYNC_DW=1" bash tools/gpu_ab_env.sh'
# each case is one env assignment (or several joined by commas); REPS runs per case,
# interleaved (A B A B ...) so box drift hits both alike.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
O=gpurun_out/abenv
mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  for c in $CASES; do
    tag=$(echo $c | tr ',=/.' '____')
    env $(echo $c | tr ',' ' ') timeout -k 10 300 python -u bench.py --cpu-baseline 0 ${BENCH_ARGS} > $O/${tag}_$r.log 2>&1 || { tail -20 $O/${tag}_$r.log; exit 1; }
    echo "$c run $r: $(python3 -c "import json; d=json.loads(open('$O/${tag}_$r.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
