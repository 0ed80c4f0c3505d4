#!/bin/bash
# PMC passes over the encoder's four GEMM roles (current default variants), one pass per
# counter group (rocprofv3 does not split counters over passes).
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc; mkdir -p $OUT
CASES=${CASES:-"12800,2304,768,0,298;12800,768,768,0,282;12800,3072,768,1,213;12800,768,3072,0,282"}
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 120 python3 $ROOT/tools/gemm_multi.py "$CASES" 20 > $OUT/timing.txt 2>&1 || exit 1
i=0
for P in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TA_BUSY_avr" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 $ROOT/tools/gemm_multi.py "$CASES" 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo pmc-done
