# Same-box A/B of the ensemble's concurrency: hipGraph vs eager, four member streams vs in order.
#   gpurun -- 'bash tools/ens_streams_ab.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-ens_streams}
mkdir -p $OUT
cd $ROOT
for i in $(seq 1 ${REPS:-2}); do
  for s in "g1s1:1:1" "g1s0:1:0" "g0s1:0:1" "g0s0:0:0"; do
    IFS=: read name g st <<< "$s"
    SGCN_ENS_STREAMS=$st timeout -k 10 300 python bench.py --config ens --cpu-baseline 0 --roofline 0 \
      --graph-ens $g > $OUT/${name}_$i.log 2>&1 || { tail -20 $OUT/${name}_$i.log; exit 1; }
    python -c "
import json
d=json.loads(open('$OUT/${name}_$i.log').read().strip().splitlines()[-1])
print('$name graph=$g streams=$st', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
  done
done
