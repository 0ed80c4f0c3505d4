#!/bin/bash
# Round 5: the LayerNorm fold on the 24-bit residual stream — parity tests, then the same-box
# A/B against the shipped default and the fp32-x fold. Output under gpurun_out/r05_fold/.
set -o pipefail
out=gpurun_out/r05_fold
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "lnfold or cls_prune_and_deferred or blocked_u_is_bit_identical" -s > $out/parity.log 2>&1 \
  || { echo "parity failed"; tail -40 $out/parity.log; exit 1; }
grep -E "passed|failed|rel |err " $out/parity.log | tail -30
bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--tuning lnfold=1" "--tuning lnfold=1;x24=0" \
  > $out/ab.log 2>&1 || { echo "A/B failed"; tail -20 $out/ab.log; exit 1; }
cat $out/ab.log
