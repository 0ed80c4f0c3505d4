#!/bin/bash
# r04 second session: QKV on the persistent ping-pong (column-group-major map) against the shipped
# 240x256 tile, bs 256 fp16, alternating
set -o pipefail
bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "--tuning qkv_pp=1" || exit 1
