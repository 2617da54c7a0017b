# dW tile microbenchmark (tools/bench/dwbench, built in-tree beforehand) on the GPU box:
#   gpurun -- 'TAG=r05_dw [MODES="64 b h"] bash tools/gpu_dwbench.sh'
#   modes: 64 = the 64 x 64 shapes, b = 128 x 128, h = the 256-row split-count sweep
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-dwbench}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for m in ${MODES:-64 b}; do
  arg=$m; [ $m = 64 ] && arg=""
  timeout -k 10 240 ./tools/bench/dwbench $arg > $OUT/dw_$m.txt 2>&1 || { tail -20 $OUT/dw_$m.txt; exit 1; }
  cat $OUT/dw_$m.txt
done
