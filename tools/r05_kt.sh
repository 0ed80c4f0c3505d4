#!/bin/bash
# Kernel-trace stats of the default bench against tuning arms (per-kernel average durations).
#   bash tools/r05_kt.sh OUTDIR "<tuning spec>" ...   ("-" = the shipped default)
set -e
OUT=$1; shift
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for arm in "$@"; do
  X=()
  [ "$arm" != "-" ] && X=(--tuning "$arm")
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/kt$i" -o run \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline "${X[@]}" > "$ROOT/$OUT/kt$i.log" 2>&1
  echo "arm $i: $arm" >> "$ROOT/$OUT/arms.txt"
  i=$((i+1))
done
echo kt-done
