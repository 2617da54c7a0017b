# Runs GPU steps in order, each under its own time limit; continues past an ordinary
# failure (e.g. a failing test) but stops at a time limit, kill, abort or fault
# (rc 124/137/134/139 or > 128). Usage (on the GPU box):
#   bash tools/gpu_steps.sh OUTDIR "SECONDS|name|command" ...
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/$1; shift
mkdir -p $OUT
cd $ROOT
for step in "$@"; do
  lim=${step%%|*}; rest=${step#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($lim s): $cmd" | tee -a $OUT/steps.txt
  timeout -k 10 $lim bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  echo "   rc=$rc" | tee -a $OUT/steps.txt
  tail -4 $OUT/$name.log
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc $rc)" | tee -a $OUT/steps.txt; exit $rc; fi
done
echo STEPS_DONE
