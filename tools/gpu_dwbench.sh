# dW tile microbenchmark (tools/bench/dwbench, built in-tree beforehand) on the GPU box:
#   gpurun -- 'TAG=r05_dw bash tools/gpu_dwbench.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-dwbench}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
timeout -k 10 180 ./tools/bench/dwbench > $OUT/dw64.txt 2>&1 || { tail -20 $OUT/dw64.txt; exit 1; }
cat $OUT/dw64.txt
timeout -k 10 240 ./tools/bench/dwbench b > $OUT/dw128.txt 2>&1 || { tail -20 $OUT/dw128.txt; exit 1; }
cat $OUT/dw128.txt
