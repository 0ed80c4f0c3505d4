#!/bin/bash
# r04 second session, GPU call 5: the blocked u / u8 layout (+ blocked MX scales), committed
# at the end of the first session without a speed A/B: shipped vs u_blocked=0, config 5 and the
# bs-256 fp16 headline, alternating on one box
set -o pipefail
for r in 1 2; do
  bash tools/ab_envs.sh "--dtype mxfp8 --batch 512" 1 - "--tuning u_blocked=0" || exit 1
  bash tools/ab_envs.sh "--steps 20 --warmup 5" 1 - "--tuning u_blocked=0" || exit 1
done
bash tools/ab_envs.sh "--dtype bf16 --batch 512" 1 - || exit 1
