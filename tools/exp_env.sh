#!/bin/bash
# In-model A/B of environment settings: each argument is a space-separated list of VAR=value
# assignments (e.g. "CLIPVIT_CLS_PRUNE=0"), run twice in alternation.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for E in "$@"; do
    env $E timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/env_b.log 2>&1 || { echo "bench failed $E"; tail gpurun_out/env_b.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/env_b.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('$E', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['model_mfma_frac'], {k:round(v,3) for k,v in f.items()})"
  done
done
