#!/bin/bash
# add_layernorm with two rows per wave (CLIPVIT_LN_RPW=2) against one (=1, default):
# bit-identity test first, then the in-model A/B of tools/exp_env.sh (layernorm family).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "bit_identical" > gpurun_out/lnrpw_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/lnrpw_tests.log; exit 1; }
tail -2 gpurun_out/lnrpw_tests.log
bash tools/exp_env.sh "CLIPVIT_LN_RPW=2" "CLIPVIT_LN_RPW=1"
