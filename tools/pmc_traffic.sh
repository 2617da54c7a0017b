# HBM traffic per kernel from rocprofv3 PMC counters (MI355X_MICROARCH.md §HBM):
# FETCH_SIZE and WRITE_SIZE in SEPARATE passes (TCC slots), kernel-trace only.
# Usage (on the GPU box): bash tools/pmc_traffic.sh <outdir> [bench args...]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/$OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $C --kernel-trace --output-format csv \
    -d $ROOT/$OUT/$C -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 \
    --cpu-baseline 0 --roofline 0 "$@" > $ROOT/$OUT/$C.log 2>&1
done
