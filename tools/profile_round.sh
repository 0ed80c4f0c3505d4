#!/bin/bash
# Profile the default bench command on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats      -> per-kernel average durations
#   2. rocprofv3 --pmc FETCH_SIZE            -> HBM read bytes per dispatch  (own pass)
#   3. rocprofv3 --pmc WRITE_SIZE            -> HBM write bytes per dispatch (own pass)
# Summaries are produced afterwards by tools/summarize_profiles.py into profiles/.
set -e
OUT=${1:-gpurun_out/prof}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/kt" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --profile-iters 2 > "$ROOT/$OUT/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/fetch" -o run \
  -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --profile-iters 1 > "$ROOT/$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/$OUT/write" -o run \
  -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --profile-iters 1 > "$ROOT/$OUT/write.log" 2>&1
echo profile-done
