# Same-box A/B of env-knob settings of the in-tree library, interleaved REPS times:
#   gpurun -- 'TAG=r04_ens BENCH_ARGS="--config ens" REPS=2 \
#              SETS="base: nofold:SGCN_EVAL_FOLD=0" \
#              bash tools/gpu_envab.sh'
# A set is name:VAR=V,VAR=V (empty after the colon = defaults).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-envab}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for i in $(seq 1 ${REPS:-2}); do
  for s in ${SETS}; do
    name=${s%%:*}
    envs=${s#*:}
    envp=${envs//,/ }
    env $envp timeout -k 10 300 python $ROOT/bench.py --cpu-baseline 0 ${BENCH_ARGS} > $OUT/${name}_$i.log 2>&1 || { tail -20 $OUT/${name}_$i.log; exit 1; }
    python -c "
import json
d=json.loads(open('$OUT/${name}_$i.log').read().strip().splitlines()[-1])
r=d['roofline'] or {}
b=r.get('step_breakdown_ms') or r.get('iter_breakdown_ms') or {}
print('$name', '$envs', d['value'], d['ms_per_step'], {k: v for k, v in b.items()})" | tee -a $OUT/summary.txt
  done
done
echo ENVAB_DONE
