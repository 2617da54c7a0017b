# One build->measure iteration on the GPU box (run from the repo root via gpurun):
#   gpu tests, a bench line, a kernel-trace profile (+ optional PMC traffic passes).
# Env: TESTS=<pytest -k expr | all | none>  PMC=1  BENCH_ARGS="..."  TAG=name
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
TAG=${TAG:-iter}
O=gpurun_out/$TAG
mkdir -p $O
if [ "${TESTS:-all}" != "none" ]; then
  K=""
  [ "${TESTS:-all}" != "all" ] && K="-k ${TESTS}"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $K > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
timeout -k 10 300 python -u bench.py --cpu-baseline 0 ${BENCH_ARGS} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$O/prof -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline 0 ${BENCH_ARGS} > $ROOT/$O/prof.log 2>&1
if [ "${PMC:-0}" = "1" ]; then
  cd $ROOT && bash tools/pmc_traffic.sh $O/pmc ${BENCH_ARGS}
fi
echo DONE
