# Over-fetch attribution of the forward contraction (verdict r03 weak #2), on the GPU box:
#   bash tools/gpu_ofetch.sh [outdir]    (binaries prebuilt here: tools/build_ofetch.sh)
# Per build variant: one timing run, then one rocprofv3 PMC pass per counter set
# (kernel-trace only, each under its own time limit).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/${1:-gpurun_out/r04_ofetch}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
for b in ${BINS:-prod d1 d2 xnt asc1}; do
  BIN=$ROOT/tools/bench/bin/ofetch_$b
  timeout -k 10 120 $BIN > $OUT/time_$b.txt 2>&1
  i=0
  for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    i=$((i+1))
    ok=1
    for c in $P; do grep -q "${c%_sum}" $OUT/avail.txt || ok=0; done
    if [ $ok = 0 ]; then echo "skip $P" >> $OUT/skipped.txt; continue; fi
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv \
      -d $OUT/$b/p$i -o run -- $BIN > $OUT/$b.p$i.log 2>&1
  done
  echo "variant $b done"
done
echo OFETCH_DONE
