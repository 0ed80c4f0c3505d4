#!/bin/bash
# Round 5: per-role kernel trace + FETCH_SIZE / WRITE_SIZE passes of the shipped default and of
# the LayerNorm fold on the 24-bit stream (tuning lnfold=1), same box. Summaries are made on the
# host: python tools/summarize_profiles.py gpurun_out/r05_foldprof/<arm> r05_fold_<arm> 256 --summary-only
set -e
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for arm in def fold; do
  OUT=$ROOT/gpurun_out/r05_foldprof/$arm
  mkdir -p $OUT
  X=(); [ $arm = fold ] && X=(--tuning lnfold=1)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run \
    -- python3 $ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --profile-iters 2 "${X[@]}" > $OUT/kt.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run \
    -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --profile-iters 1 "${X[@]}" > $OUT/fetch.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run \
    -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --profile-iters 1 "${X[@]}" > $OUT/write.log 2>&1
  echo "$arm done"
done
