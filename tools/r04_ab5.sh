#!/bin/bash
# r04 second session, GPU call 6: the persistent MX / 16-bit tiles with blocked A / C as
# compile-time parameters (the runtime flags had spilled the MX c_fc accumulators into scratch,
# reloaded under vmcnt(0) in the k-loop). MX + kernel tests, then config 5 (blocked vs row-major
# u8) and the bs-256 fp16 line, alternating, with bf16 bs 512 for the ratio
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_mx8.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/k_tests.log 2>&1 \
  || { tail -30 gpurun_out/k_tests.log; exit 1; }
tail -2 gpurun_out/k_tests.log
for r in 1 2; do
  bash tools/ab_envs.sh "--dtype mxfp8 --batch 512" 1 - "--tuning u_blocked=0" || exit 1
  bash tools/ab_envs.sh "--dtype bf16 --batch 512" 1 - || exit 1
  bash tools/ab_envs.sh "--steps 20 --warmup 5" 1 - || exit 1
done
