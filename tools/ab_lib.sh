# Same-box A/B of the working tree's library against a build of another commit:
#   bash tools/ab_lib.sh <commit>          (here: builds tools/ab/libshiftgcn_hip_base.so)
#   gpurun -- 'bash tools/ab_lib.sh run'   (there: alternating bench runs, base vs tree)
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
if [ "$1" != "run" ]; then
  rm -rf /tmp/sgcn_ab && mkdir -p /tmp/sgcn_ab $ROOT/tools/ab
  git -C $ROOT archive ${1:-HEAD} shift-gcn_amd/csrc include | tar -x -C /tmp/sgcn_ab
  make -C /tmp/sgcn_ab/shift-gcn_amd/csrc -j8 OUT=$ROOT/tools/ab/libshiftgcn_hip_base.so > /dev/null
  echo built tools/ab/libshiftgcn_hip_base.so from ${1:-HEAD}
  exit 0
fi
mkdir -p $ROOT/gpurun_out/ab
for i in 1 2; do
  for v in base tree; do
    if [ $v = base ]; then export SGCN_LIB_PATH=$ROOT/tools/ab/libshiftgcn_hip_base.so; else unset SGCN_LIB_PATH; fi
    timeout -k 10 300 python $ROOT/bench.py --cpu-baseline 0 > $ROOT/gpurun_out/ab/$v$i.json
    python -c "import json;d=json.loads(open('$ROOT/gpurun_out/ab/$v$i.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'])" | tee -a $ROOT/gpurun_out/ab/summary.txt
  done
done
