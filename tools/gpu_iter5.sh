# Round-5 iteration check in ONE gpurun call: the GPU suite (or a -k subset), then the
# NTU / MP / ENS bench lines (no CPU baseline), logs under gpurun_out/$TAG.
#   gpurun -- 'TAG=r05a [K="expr"] [NOBENCH=1] bash tools/gpu_iter5.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-iter}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
KA=()
if [ -n "$K" ]; then KA=(-k "$K"); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "${KA[@]}" > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
if [ -n "$NOBENCH" ]; then exit 0; fi
for c in ntu mp ens; do
  timeout -k 10 300 python -u bench.py --cpu-baseline 0 --config $c > $OUT/bench_$c.log 2>&1 || { tail -20 $OUT/bench_$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_$c.log').read().strip().splitlines()[-1]); print('$c', d['value'], d['unit'], d['roofline']['frac'] if d['roofline'] else None)"
done
