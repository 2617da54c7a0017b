# FETCH_SIZE calibration by access shape (tools/bench/fetchcal): timing + one PMC pass per shape set
#   gpurun -- 'TAG=r03b bash tools/gpu_fetchcal.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${TAG:-fetchcal}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for S in "128 384 3750" "128 384 4096" "64 192 7500"; do
  tag=$(echo $S | tr ' ' '_')
  timeout -k 10 60 $ROOT/tools/bench/fetchcal $S all > $OUT/time_$tag.txt 2>&1
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc_${tag}/$C -o run -- $ROOT/tools/bench/fetchcal $S all > $OUT/pmc_${tag}_$C.log 2>&1
  done
  echo "$S done"
done
