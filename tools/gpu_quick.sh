# Quick GPU check: the gpu test suite (or a -k subset) + one bench line.
#   gpurun -- 'K="expr" bash tools/gpu_quick.sh'   (K unset -> all gpu tests)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out/q
KA=()
if [ -n "$K" ]; then KA=(-k "$K"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${KA[@]}" > gpurun_out/q/tests.log 2>&1 || { tail -40 gpurun_out/q/tests.log; exit 1; }
tail -2 gpurun_out/q/tests.log
timeout -k 10 300 python -u bench.py --cpu-baseline 0 ${BENCH_ARGS} > gpurun_out/q/bench.log 2>&1 || { tail -20 gpurun_out/q/bench.log; exit 1; }
tail -1 gpurun_out/q/bench.log
