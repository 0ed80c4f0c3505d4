#!/bin/bash
# MX-fp8 (config 5) tile A/B on the bench: QKV, out_proj, c_fc, c_proj variant sets.
set -o pipefail
bash tools/ab_envs.sh "--dtype mxfp8 --batch 512 --steps 20" 3 "CLIPVIT_MX8_VARIANTS=2,2,2,2" "-" "CLIPVIT_MX8_VARIANTS=3,3,2,3" "CLIPVIT_MX8_VARIANTS=3,2,3,3"
