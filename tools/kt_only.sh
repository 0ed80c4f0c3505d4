#!/bin/bash
# Kernel-trace pass only (per-kernel average durations) of a bench command, on the GPU box:
#   bash tools/kt_only.sh OUT_DIR "<bench args>"
set -e
OUT=${1:-gpurun_out/kt}
ARGS=${2:-}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --profile-iters 2 $ARGS > "$ROOT/$OUT.log" 2>&1
echo kt-done
