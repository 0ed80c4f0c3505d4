#!/bin/bash
# PMC passes over the bench's forward (in-model kernel behaviour: clock, MFMA busy, L2 hit rate).
set -o pipefail
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmcm; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-iters 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo pmc-done
