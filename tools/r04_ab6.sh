#!/bin/bash
# r04 second session, GPU call 7: MX c_fc row split re-measured on the spill-free MX tiles
set -o pipefail
for r in 1 2; do
  bash tools/ab_envs.sh "--dtype mxfp8 --batch 512" 1 - "--tuning mx8_split_tail=2" || exit 1
done
bash tools/ab_envs.sh "--dtype bf16 --batch 512" 1 - || exit 1
