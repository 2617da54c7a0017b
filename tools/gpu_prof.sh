# rocprofv3 kernel-trace stats of a short bench run: gpurun -- 'TAG=x bash tools/gpu_prof.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-prof}
mkdir -p $ROOT/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/$TAG/prof -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --cpu-baseline 0 --roofline 0 ${BENCH_ARGS} > $ROOT/gpurun_out/$TAG/prof.log 2>&1
tail -1 $ROOT/gpurun_out/$TAG/prof.log
