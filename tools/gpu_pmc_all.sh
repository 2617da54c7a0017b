# HBM traffic per op class for every bench config (rocprofv3 FETCH_SIZE / WRITE_SIZE in
# separate kernel-trace passes, serialized schedule), raw CSVs under gpurun_out/$TAG/pmc_<cfg>;
# then locally: python tools/pmc_summary.py gpurun_out/$TAG/pmc_<cfg> --json ... --iters N
# (ntu/mp: 3 steps; ens: 5 ensemble iterations = 2 capture warm-ups + 1 + 2)
#   gpurun -- 'TAG=r03f bash tools/gpu_pmc_all.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-pmc_all}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for CFG in ${CFGS:-ntu mp ens}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    SGCN_ASYNC_DW=0 SGCN_ENS_STREAMS=0 timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv \
      -d $OUT/pmc_$CFG/$C -o run -- python3 $ROOT/bench.py --config $CFG --steps 2 --warmup 1 \
      --cpu-baseline 0 --roofline 0 > $OUT/pmc_${CFG}_$C.log 2>&1
    echo "PMC $CFG $C"
  done
done
