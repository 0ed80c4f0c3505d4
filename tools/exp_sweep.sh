#!/bin/bash
# In-model A/B of GEMM role variants: CLIPVIT_GEMM_VARIANTS strings given as arguments.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for V in "$@"; do
    CLIPVIT_GEMM_VARIANTS=$V timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/sweep_b.log 2>&1 || { echo "bench failed $V"; tail gpurun_out/sweep_b.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/sweep_b.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('$V', d['value'], d['ms_per_step'], {k:round(v,3) for k,v in f.items()})"
  done
done
