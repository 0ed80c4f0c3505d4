#!/bin/bash
# A/B of an environment knob on the bench (run on the GPU box via gpurun from the repo root):
#   bash tools/ab_env.sh "<bench args>" VAR "val1 val2" [rounds]
# alternates the values (rounds x), one bench process per run, prints value + family times.
set -o pipefail
ARGS=$1; VAR=$2; VALS=$3; R=${4:-2}
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 240 python -u bench.py $ARGS --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { echo "bench failed ($VAR=$v)"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab.json'))
f=d['roofline']['family_ms_per_forward']
print('$VAR=$v', '$ARGS', round(d['value']), 'img/s', ' '.join(f'{k}={v:.3f}' for k,v in f.items()), 'parity', d.get('parity',{}).get('max_rel_logit_err_vs_cpu_fp32_oracle'), flush=True)"
  done
done
