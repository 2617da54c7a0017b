# Forward / dW contraction microbenchmark (tools/bench/pwbench, built in-tree beforehand):
#   gpurun -- 'TAG=r05_pw MODE=fx bash tools/gpu_pwbench.sh'   (MODE: f, w, fw; x = variants)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-pwbench}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
if [ -n "${MODE#?}" ] && [ "${MODE: -1}" = x ]; then EXTRA=x; fi
timeout -k 10 400 ./tools/bench/pwbench ${MODE%x} $EXTRA > $OUT/pwbench.txt 2>&1 || { tail -20 $OUT/pwbench.txt; exit 1; }
cat $OUT/pwbench.txt
