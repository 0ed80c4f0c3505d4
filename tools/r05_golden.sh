#!/bin/bash
# Round 5: the reference-harness fixtures (flat + CLIP-scale) with the literal rank-1 rule;
# prints the per-case worst relative logit error. Output under gpurun_out/r05_golden/.
set -o pipefail
out=gpurun_out/r05_golden
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_golden.py -x -v --timeout 400 --timeout-method thread \
  -k "flat_fixtures or clipscale_harness" -s > $out/golden.log 2>&1 \
  || { echo "golden failed"; grep -E "rel logit|swaps|Error|assert" $out/golden.log | tail -30; exit 1; }
grep -E "rel logit|swaps|argmax|passed|failed" $out/golden.log
