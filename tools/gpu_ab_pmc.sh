# One GPU call for a library change: GPU tests (a -k/-file subset), same-box A/B of the tree's
# library against tools/ab/libshiftgcn_hip_base.so (bash tools/ab_lib.sh <commit> first), and
# the tree's HBM traffic (FETCH_SIZE / WRITE_SIZE passes, serialized schedule).
#   gpurun -- 'TAG=r03a TESTS="tests/test_gpu_kernels.py" bash tools/gpu_ab_pmc.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-ab}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
if [ "${AB:-1}" = "1" ]; then
  for i in $(seq 1 ${REPS:-2}); do
    for v in base tree; do
      if [ $v = base ]; then export SGCN_LIB_PATH=$ROOT/tools/ab/libshiftgcn_hip_base.so; else unset SGCN_LIB_PATH; fi
      timeout -k 10 300 python $ROOT/bench.py --cpu-baseline 0 ${BENCH_ARGS} > $OUT/${v}$i.log 2>&1 || { tail -20 $OUT/${v}$i.log; exit 1; }
      python -c "import json;d=json.loads(open('$OUT/${v}$i.log').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],d['roofline']['step_breakdown_ms'] if d['roofline'] else '')" | tee -a $OUT/summary.txt
    done
  done
  unset SGCN_LIB_PATH
fi
if [ "${PMC:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  for C in FETCH_SIZE WRITE_SIZE; do
    SGCN_ASYNC_DW=0 timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc/$C -o run \
      -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --roofline 0 ${BENCH_ARGS} > $OUT/pmc_$C.log 2>&1
    echo PMC_$C
  done
fi
echo DONE
