#!/bin/bash
# r06 session 2: tile / split choices re-checked at the sc0 sc1 store policy (B/32 bs 256, same box,
# 3 alternations): QKV on the balanced grid (v75), c_fc as the row split (v62 + v81), the two-lane
# split at bs 256
set -o pipefail
O=gpurun_out/c17
mkdir -p $O
bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "--tuning qkv_variant=75" "--tuning fc_balanced=0" "--tuning split_min=256" > $O/tune_ab.log 2>&1
cat $O/tune_ab.log
