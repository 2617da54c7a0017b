# One GPU call for a streaming-kernel change: a GPU test subset, the isolated shift-backward
# probe (tools/bench/gbn_probe.py) on the base library and the tree, and a same-box bench
# A/B (base = tools/ab/libshiftgcn_hip_base.so, built by `bash tools/ab_lib.sh <commit>`).
#   gpurun -- 'TAG=r03x TESTS="tests/test_gpu_tshift.py" bash tools/gpu_probe.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-probe}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
# extra variants: tools/ab/libshiftgcn_hip_<name>.so for each name in $VARIANTS
for shape in ${PROBE_SHAPES:-64:300 128:150 256:75}; do
  for v in tree $VARIANTS; do
    if [ $v = tree ]; then unset SGCN_LIB_PATH; else export SGCN_LIB_PATH=$ROOT/tools/ab/libshiftgcn_hip_$v.so; fi
    timeout -k 10 120 python -u tools/bench/gbn_probe.py ${shape/:/ } > $OUT/probe_${v}_${shape/:/_}.txt 2>&1 || { cat $OUT/probe_${v}_${shape/:/_}.txt; exit 1; }
    echo "$v $(tail -1 $OUT/probe_${v}_${shape/:/_}.txt)" | tee -a $OUT/probe.txt
  done
done
unset SGCN_LIB_PATH
if [ "${AB:-1}" = "1" ]; then
  for i in $(seq 1 ${REPS:-2}); do
    for v in base tree; do
      if [ $v = base ]; then export SGCN_LIB_PATH=$ROOT/tools/ab/libshiftgcn_hip_base.so; else unset SGCN_LIB_PATH; fi
      timeout -k 10 300 python $ROOT/bench.py --cpu-baseline 0 ${BENCH_ARGS} > $OUT/${v}$i.log 2>&1 || { tail -20 $OUT/${v}$i.log; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/${v}$i.log').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['roofline']['step_breakdown_ms'] if d['roofline'] else '')" | tee -a $OUT/summary.txt
    done
  done
fi
echo DONE
