#!/bin/bash
# r04 second session, GPU call 4: MX-fp8 c_fc whole-round row split (tests, then config-5 A/B
# against one launch and the 160x128 tail, with bf16 bs 512 lines for the ratio)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx8.py -x -q --timeout 300 --timeout-method thread > gpurun_out/mx8_tests.log 2>&1 \
  || { tail -30 gpurun_out/mx8_tests.log; exit 1; }
tail -3 gpurun_out/mx8_tests.log
for r in 1 2; do
  bash tools/ab_envs.sh "--dtype mxfp8 --batch 512" 1 - "--tuning mx8_split_tail=0" "--tuning mx8_split_tail=5" || exit 1
  bash tools/ab_envs.sh "--dtype bf16 --batch 512" 1 - || exit 1
done
