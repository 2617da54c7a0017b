# VGPR / AGPR / LDS / spill counts of every gfx950 kernel in an in-tree object file:
#   bash tools/kernel_regs.sh shift-gcn_amd/csrc/build/tshift.o [name-filter]
set -e
O=$1
T=$(mktemp -d)
L=/opt/rocm/lib/llvm/bin
$L/llvm-objcopy --dump-section=.hip_fatbin=$T/fb "$O"
$L/clang-offload-bundler --unbundle --type=o --input=$T/fb --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/co
$L/llvm-readelf --notes $T/co | python3 -c "
import sys, re, subprocess
txt = sys.stdin.read()
flt = sys.argv[1] if len(sys.argv) > 1 else ''
for blk in re.split(r'\n  - ', txt):
    m = re.search(r'\.name:\s+(\S+)', blk)
    if not m or m.group(1).endswith('.kd'):
        continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\S+)', blk) or [None, '?'])[1]
    name = subprocess.run(['c++filt', m.group(1)], capture_output=True, text=True).stdout.strip()
    if flt and flt not in name:
        continue
    print(f\"vgpr {g('vgpr_count'):>4} agpr {g('agpr_count'):>4} lds {g('group_segment_fixed_size'):>6} spill {g('vgpr_spill_count'):>3}  {name[:170]}\")
" "${2:-}"
rm -rf $T
