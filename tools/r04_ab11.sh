#!/bin/bash
# r04 closing session: head products on 32-column workgroups (tuning head_cols=32: 2x the
# workgroups of cls_ln_proj / logits) — bit-identity test, head tests, then the same-box A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -q --timeout 200 --timeout-method thread -k "head_column or classify_matches or golden or harness" > gpurun_out/ab11_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/ab11_tests.log; exit 1; }
tail -1 gpurun_out/ab11_tests.log
bash tools/ab_envs.sh "" 3 - "--tuning head_cols=32"
