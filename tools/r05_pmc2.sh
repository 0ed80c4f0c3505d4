#!/bin/bash
# Round 5: LDS / instruction-issue PMC passes of variant 72 (QKV shape, row-major and blocked
# operands) and the v62 copy. Output under gpurun_out/r05_pmc2/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
out=$R/gpurun_out/r05_pmc2
mkdir -p $out
for kind in 0 1 2; do
  P="$R/tools/probes/gemm_probe p32run 12800 2304 768 0 0 30 $kind"
  i=0
  for set in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
             "SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $out/k$kind/p$i -o run -- $P > $out/k$kind.p$i.log 2>&1 \
      || { rc=$?; echo "kind $kind pass $i ($set) failed rc=$rc"; tail -3 $out/k$kind.p$i.log; [ $rc -ge 124 ] && exit 1; }
  done
done
echo done
