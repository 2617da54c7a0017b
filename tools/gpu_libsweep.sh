# Same-box sweep of several library builds against the base (tools/ab/lib_<name>.so, built
# from copies of csrc with different -D knobs), interleaved, REPS rounds, one config:
#   gpurun -- 'TAG=r05_nt2 LIBS="epi bna side" CONFIG=ntu REPS=2 bash tools/gpu_libsweep.sh'
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-libsweep}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for i in $(seq 1 ${REPS:-2}); do
  for v in base ${LIBS}; do
    if [ $v = base ]; then L=$ROOT/tools/ab/libshiftgcn_hip_base.so; else L=$ROOT/tools/ab/lib_$v.so; fi
    SGCN_LIB_PATH=$L timeout -k 10 300 python -u bench.py --cpu-baseline 0 --config ${CONFIG:-ntu} > $OUT/${v}_$i.log 2>&1 || { tail -20 $OUT/${v}_$i.log; exit 1; }
    python -c "
import json
d=json.loads(open('$OUT/${v}_$i.log').read().strip().splitlines()[-1])
cr=d['roofline']['class_rates'] if d['roofline'] else {}
print('${CONFIG:-ntu} $v$i', d['value'], d['ms_per_step'], ' '.join(f'{k}={v[\"ms\"]}' for k, v in cr.items()))" | tee -a $OUT/summary.txt
  done
done
