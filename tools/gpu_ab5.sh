# Same-box A/B of the tree's library against tools/ab/libshiftgcn_hip_base.so (built by
# `bash tools/ab_lib.sh <commit>`), REPS interleaved rounds per config in CONFIGS:
#   gpurun -- 'TAG=r05_ab CONFIGS="ntu mp" REPS=3 bash tools/gpu_ab5.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-ab5}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for c in ${CONFIGS:-ntu}; do
  for i in $(seq 1 ${REPS:-2}); do
    for v in base tree; do
      if [ $v = base ]; then export SGCN_LIB_PATH=$ROOT/tools/ab/libshiftgcn_hip_base.so; else unset SGCN_LIB_PATH; fi
      timeout -k 10 300 python -u bench.py --cpu-baseline 0 --config $c ${BENCH_ARGS} > $OUT/${c}_${v}$i.log 2>&1 || { tail -20 $OUT/${c}_${v}$i.log; exit 1; }
      python -c "
import json
d=json.loads(open('$OUT/${c}_${v}$i.log').read().strip().splitlines()[-1])
cr=d['roofline']['class_rates'] if d['roofline'] else {}
print('$c $v$i', d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"ms\"]}' for k, v in cr.items()))" | tee -a $OUT/summary.txt
    done
  done
done
