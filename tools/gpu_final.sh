# Round artifacts on the GPU box: gpurun -- 'TAG=r02g bash tools/gpu_final.sh'
#   GPU tests (TESTS=0 skips), bench lines NTU (with CPU baseline) / MP / ENS, the rocprofv3
#   kernel-trace stats of the NTU bench command, and of the same command serialized
#   (SGCN_ASYNC_DW=0: the schedule bench.py's roofline steps use). PMC=1: HBM traffic passes.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-final}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
fi
timeout -k 10 400 python -u bench.py > $OUT/bench_ntu.log 2>&1 || { tail -20 $OUT/bench_ntu.log; exit 1; }
tail -1 $OUT/bench_ntu.log > $OUT/bench_ntu.json
echo "NTU $(cut -c1-120 $OUT/bench_ntu.json)"
timeout -k 10 400 python -u bench.py --config mp > $OUT/bench_mp.log 2>&1 || { tail -20 $OUT/bench_mp.log; exit 1; }
tail -1 $OUT/bench_mp.log > $OUT/bench_mp.json
echo "MP $(cut -c1-120 $OUT/bench_mp.json)"
timeout -k 10 400 python -u bench.py --config ens > $OUT/bench_ens.log 2>&1 || { tail -20 $OUT/bench_ens.log; exit 1; }
tail -1 $OUT/bench_ens.log > $OUT/bench_ens.json
echo "ENS $(cut -c1-120 $OUT/bench_ens.json)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
  -- python3 $ROOT/bench.py --cpu-baseline 0 > $OUT/prof.log 2>&1
echo "PROF $(tail -1 $OUT/prof.log | cut -c1-100)"
SGCN_ASYNC_DW=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_serial -o run \
  -- python3 $ROOT/bench.py --cpu-baseline 0 > $OUT/prof_serial.log 2>&1
echo "PROF_SERIAL $(tail -1 $OUT/prof_serial.log | cut -c1-100)"
if [ "${PMC:-0}" = "1" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    SGCN_ASYNC_DW=0 timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc/$C -o run \
      -- python3 $ROOT/bench.py --steps 2 --warmup 1 --cpu-baseline 0 --roofline 0 > $OUT/pmc_$C.log 2>&1
    echo PMC_$C
  done
fi
echo DONE
