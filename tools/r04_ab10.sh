#!/bin/bash
# r04 closing session: class-token tail GEMM tile (tuning tail_variant): 90 (64x64, shipped)
# against 81 (128x128) and 22 (160x128), same box
set -o pipefail
bash tools/ab_envs.sh "" 2 - "--tuning tail_variant=81" "--tuning tail_variant=22"
