# Builds the over-fetch probe variants (tools/bench/ofetch.hip) into tools/bench/bin/.
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17"
S=$ROOT/tools/bench/ofetch.hip
mkdir -p $ROOT/tools/bench/bin
$H $S -o $ROOT/tools/bench/bin/ofetch_prod &
$H -DSGCN_PW_DIAG=1 $S -o $ROOT/tools/bench/bin/ofetch_d1 &
$H -DSGCN_PW_DIAG=2 $S -o $ROOT/tools/bench/bin/ofetch_d2 &
$H -DSGCN_PW_XPOL=2 $S -o $ROOT/tools/bench/bin/ofetch_xnt &
$H -DSGCN_PW_APOL=16 $S -o $ROOT/tools/bench/bin/ofetch_asc1 &
$H -DSGCN_PW_XCD=0 $S -o $ROOT/tools/bench/bin/ofetch_noxcd &
wait
ls -la $ROOT/tools/bench/bin/ofetch_*
