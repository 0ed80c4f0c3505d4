#!/bin/bash
# r05: blocked weight copy on the persistent ping-pong tile (v62/63): kernel screens + same-box A/B
# against the previous default (blocked W on the pipelined and 32-deep tiles only).
set -o pipefail
out=gpurun_out/r05_v62blk
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -m gpu -k "race_screen or blocked or gemm_shapes" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "--tuning w_blocked=1" > $out/b32.log 2>&1 || { echo "b32 A/B failed"; tail -5 $out/b32.log; exit 1; }
bash tools/ab_envs.sh "--model ViT-B/16 --steps 10 --warmup 3" 2 - "--tuning w_blocked=1" > $out/b16.log 2>&1 || { echo "b16 A/B failed"; exit 1; }
cat $out/b32.log $out/b16.log | cut -c1-140
