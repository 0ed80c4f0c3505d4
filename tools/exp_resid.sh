#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread -k "parity or golden" > gpurun_out/resid_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/resid_tests.log; exit 1; }
grep -E "rel logit|passed|failed" gpurun_out/resid_tests.log | tail -20
for r in 1 2; do
  for M in 0 1; do
    CLIPVIT_RESID16=$M timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/resid_b.log 2>&1 || { echo "bench failed"; tail gpurun_out/resid_b.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/resid_b.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('resid16=$M', d['value'], d['ms_per_step'], {k:round(v,3) for k,v in f.items()})"
  done
done
