set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
mkdir -p gpurun_out/bs
for B in 64 32 16 8; do
  timeout -k 10 200 python -u bench.py --cpu-baseline 0 --batch $B --steps 20 > gpurun_out/bs/b$B.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/bs/b$B.log').read().strip().splitlines()[-1]);r=d['roofline'];print($B,d['value'],d['ms_per_step'],r['step_ms_event_timed'],{k:round(v/$B*64,3) for k,v in r['step_breakdown_ms'].items()})"
done
