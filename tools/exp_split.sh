#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for S in 0 128; do
    CLIPVIT_SPLIT_MIN=$S timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/split_b.log 2>&1 || { echo "bench failed"; tail gpurun_out/split_b.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/split_b.log').read().strip().splitlines()[-1])
print('split=$S', d['value'], d['ms_per_step'])"
  done
done
