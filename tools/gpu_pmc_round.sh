# One profiling round on the GPU box (each rocprofv3 pass its own process and time limit):
#   gpurun -- 'TAG=r02f bash tools/gpu_pmc_round.sh'
# 1. kernel-trace --stats of a 5-step bench run; 2. FETCH_SIZE / WRITE_SIZE passes
# (HBM traffic, tools/pmc_summary.py); 3. one SQ pass with the MFMA-busy counters
# (tools/mfma_summary.py).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r02f}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
  -- python3 $ROOT/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline 0 > $OUT/prof.log 2>&1
echo PROF_DONE
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc/$C -o run \
    -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --roofline 0 > $OUT/pmc_$C.log 2>&1
  echo PMC_$C
done
timeout -k 10 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d $OUT/sq -o run \
  -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --roofline 0 > $OUT/sq.log 2>&1
echo SQ_DONE
