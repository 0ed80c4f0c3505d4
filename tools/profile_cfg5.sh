#!/bin/bash
# BASELINE config 5 (MX-fp8 Linears, bs 512) under rocprofv3 on the GPU box: kernel trace, then
# the MFMA-busy / wait and L2 counter passes (one rocprofv3 run each), then the summary
# (tools/summarize_cfg5.py; re-run it here on the merged gpurun_out/ to commit).
#   bash tools/profile_cfg5.sh OUTDIR TAG
set -e
OUT=${1:-gpurun_out/cfg5prof}
TAG=${2:-rXX}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="--dtype mxfp8 --batch 512 --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/kt" -o run \
  -- python3 "$ROOT/bench.py" $A --steps 5 --warmup 2 --profile-iters 2 > "$ROOT/$OUT/kt.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d "$ROOT/$OUT/mfma" -o run \
  -- python3 "$ROOT/bench.py" $A --steps 2 --warmup 1 --profile-iters 1 > "$ROOT/$OUT/mfma.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$ROOT/$OUT/l2" -o run \
  -- python3 "$ROOT/bench.py" $A --steps 2 --warmup 1 --profile-iters 1 > "$ROOT/$OUT/l2.log" 2>&1
cd "$ROOT"
python3 tools/summarize_cfg5.py "$OUT" "$TAG" > "$OUT/summary.log"
echo cfg5-profile-done
