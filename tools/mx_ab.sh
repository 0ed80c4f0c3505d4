#!/bin/bash
# MX-fp8 (config 5) tile A/B on the bench: QKV, out_proj, c_fc, c_proj variant sets.
set -o pipefail
bash tools/ab_envs.sh "--dtype mxfp8 --batch 512 --steps 20" 3 "--tuning mx8_variants=2,2,2,2" "-" "--tuning mx8_variants=3,3,2,3" "--tuning mx8_variants=3,2,3,3"
