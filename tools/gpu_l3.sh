# L3-order microbenchmark + FETCH/WRITE_SIZE calibration (gpurun -- bash tools/gpu_l3.sh)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/l3
mkdir -p $O
timeout -k 10 120 $ROOT/tools/bench/l3order > $O/l3order.txt 2>&1
cat $O/l3order.txt
cd /tmp && export TMPDIR=/tmp
for lane in 4 16; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib_f$lane -o run -- $ROOT/tools/bench/l3order calib $lane > $O/calib_f$lane.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/calib_w$lane -o run -- $ROOT/tools/bench/l3order calib $lane > $O/calib_w$lane.log 2>&1
done
echo DONE
