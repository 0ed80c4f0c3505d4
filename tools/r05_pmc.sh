#!/bin/bash
# Round 5: PMC passes (one counter set per rocprofv3 run, --kernel-trace + --pmc only) of the QKV
# shape on v72 (row-major / blocked operands) and the v62 copy, and of c_proj's shipped tile
# (v82 via tools/gemm_ab.py). Output under gpurun_out/r05_pmc/<kind>/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05_pmc
mkdir -p $out
for kind in 0 1 2 cproj; do
  if [ $kind = cproj ]; then P="python3 $R/tools/gemm_ab.py 12800,768,3072,0 82 1 30"
  else P="$R/tools/probes/gemm_probe p32run 12800 2304 768 0 0 30 $kind"; fi
  i=0
  for set in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $out/k$kind/p$i -o run -- $P > $out/k$kind.p$i.log 2>&1 \
      || { rc=$?; echo "kind $kind pass $i ($set) failed rc=$rc"; tail -3 $out/k$kind.p$i.log; [ $rc -ge 124 ] && exit 1; }
  done
done
echo done
