#!/bin/bash
# Round 5: the large-M roles on variant 72 + blocked W (new default) — race screen, bit-identity
# and parity tests, then same-box A/B against the r04 large-M defaults on L/14@336, B/16 and B/32.
# Output under gpurun_out/r05_large/.
set -o pipefail
out=gpurun_out/r05_large
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -k "p32_race or blocked_w or blocked_u or L14 or l14 or large" > $out/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
OLD="--tuning w_blocked=0;large_variants=3462,3463,3463,3463"
bash tools/ab_envs.sh "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2" 2 - "$OLD" > $out/l14.log 2>&1 \
  || { echo "l14 A/B failed"; tail -5 $out/l14.log; exit 1; }
bash tools/ab_envs.sh "--model ViT-B/16 --steps 10 --warmup 3" 2 - "$OLD" > $out/b16.log 2>&1 \
  || { echo "b16 A/B failed"; tail -5 $out/b16.log; exit 1; }
bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "$OLD" > $out/b32.log 2>&1 || { echo "b32 A/B failed"; tail -5 $out/b32.log; exit 1; }
cat $out/l14.log $out/b16.log $out/b32.log | cut -c1-150
