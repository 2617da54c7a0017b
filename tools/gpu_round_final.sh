# Closing artifacts of a round in ONE gpurun call (the bench lines then quote this tree's
# own PMC traffic):
#   gpurun -- 'TAG=r04_final bash tools/gpu_round_final.sh'
# 1. tools/gpu_pmc_all.sh: FETCH_SIZE / WRITE_SIZE passes of every config (serialized);
# 2. tools/pmc_summary.py on the box -> profiles/pmc_traffic*.json (tag $TAG), copied to
#    gpurun_out/$TAG/ (the box's profiles/ does not travel back);
# 3. tools/gpu_final.sh: pytest -m gpu, bench lines NTU (CPU baseline) / MP / ENS, rocprofv3
#    kernel-trace stats of the NTU bench command, default and serialized.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-final}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
TAG=$TAG bash tools/gpu_pmc_all.sh
cd $ROOT
python tools/pmc_summary.py $OUT/pmc_ntu --iters 3 --tag $TAG --json profiles/pmc_traffic.json > $OUT/pmc_traffic_by_kernel_ntu.txt
python tools/pmc_summary.py $OUT/pmc_mp --iters 3 --tag $TAG --json profiles/pmc_traffic_mp.json > $OUT/pmc_traffic_by_kernel_mp.txt
python tools/pmc_summary.py $OUT/pmc_ens --iters 5 --tag $TAG --json profiles/pmc_traffic_ens.json > $OUT/pmc_traffic_by_kernel_ens.txt
cp profiles/pmc_traffic.json $OUT/pmc_traffic_ntu.json
cp profiles/pmc_traffic_mp.json profiles/pmc_traffic_ens.json $OUT/
echo PMC_SUMMARIES
TAG=$TAG bash tools/gpu_final.sh
