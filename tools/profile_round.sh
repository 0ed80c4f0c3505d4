#!/bin/bash
# Profile the default bench command on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats      -> per-kernel average durations
#   2. rocprofv3 --pmc FETCH_SIZE            -> HBM read bytes per dispatch  (own pass)
#   3. rocprofv3 --pmc WRITE_SIZE            -> HBM write bytes per dispatch (own pass)
#   4. rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY
#                                            -> MFMA busy, clock, wait share per dispatch (own pass)
#   5. rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -> L2 hit rate per dispatch (own pass)
#   6. tools/summarize_profiles.py (host only) -> profiles/<tag>_summary.md, <tag>_fc_traffic.json
#      (written on the box for step 7; only gpurun_out/ comes back: re-run it here on the merged
#      gpurun_out/prof to commit them)
#   7. the default bench once more, with --traffic-json of step 6 -> $OUT/bench_traffic.json
# Usage: bash tools/profile_round.sh OUTDIR TAG
set -e
OUT=${1:-gpurun_out/prof}
TAG=${2:-rXX}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/kt" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --profile-iters 2 > "$ROOT/$OUT/kt.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/fetch" -o run \
  -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --profile-iters 1 > "$ROOT/$OUT/fetch.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOT/$OUT/write" -o run \
  -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --profile-iters 1 > "$ROOT/$OUT/write.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d "$ROOT/$OUT/mfma" -o run \
  -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --profile-iters 1 > "$ROOT/$OUT/mfma.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$ROOT/$OUT/l2" -o run \
  -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --profile-iters 1 > "$ROOT/$OUT/l2.log" 2>&1
cd "$ROOT"
python3 tools/summarize_profiles.py "$OUT" "$TAG" 256 > "$OUT/summary.log"
timeout -k 10 300 python3 bench.py --traffic-json "profiles/${TAG}_fc_traffic.json" > "$OUT/bench_traffic.json" 2> "$OUT/bench_traffic.err"
echo profile-done
