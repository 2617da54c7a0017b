# Same-box A/B of several library builds on the NTU bench, interleaved REPS times:
#   VARIANTS="base tree f2ub" (tree = the in-tree library, else tools/ab/libshiftgcn_hip_<v>.so)
#   gpurun -- 'TAG=r03x VARIANTS="base f2ub" REPS=3 bash tools/gpu_abn.sh'
# ENVS="SGCN_ASYNC_DW=0" adds the same runs under those env settings.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-abn}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for i in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS:-base tree}; do
    for e in none ${ENVS}; do
      if [ $v = tree ]; then unset SGCN_LIB_PATH; else export SGCN_LIB_PATH=$ROOT/tools/ab/libshiftgcn_hip_$v.so; fi
      if [ $e = none ]; then envp=""; else envp="$e"; fi
      env $envp timeout -k 10 300 python $ROOT/bench.py --cpu-baseline 0 ${BENCH_ARGS} > $OUT/${v}_${e//=/}_$i.log 2>&1 || { tail -20 $OUT/${v}_${e//=/}_$i.log; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/${v}_${e//=/}_$i.log').read().strip().splitlines()[-1]);print('$v','$e',d['value'],d['ms_per_step'],d['roofline']['step_breakdown_ms'] if d['roofline'] else '')" | tee -a $OUT/summary.txt
    done
  done
done
unset SGCN_LIB_PATH
if [ "${SHAPES:-0}" = "1" ]; then
  SGCN_ASYNC_DW=0 timeout -k 10 200 python tools/shape_breakdown.py > $OUT/shape_breakdown_serialized.txt 2>&1
fi
echo DONE
