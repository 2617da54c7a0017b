# Run a subset of GPU tests: gpurun -- 'K="expr" bash tools/gpu_tests.sh' (files in F)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out/t
KA=()
if [ -n "$K" ]; then KA=(-k "$K"); fi
timeout -k 10 900 python -u -m pytest ${F:-tests} -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > gpurun_out/t/tests.log 2>&1 || { tail -60 gpurun_out/t/tests.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED" gpurun_out/t/tests.log | tail -40
tail -2 gpurun_out/t/tests.log
