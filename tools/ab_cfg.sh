#!/bin/bash
# A/B of whole environment settings on the bench (run on the GPU box via gpurun from the repo root):
#   bash tools/ab_cfg.sh "<bench args>" ROUNDS "SPEC1" "SPEC2" ...
# SPEC = space-separated VAR=value assignments, or "default". The specs alternate (ROUNDS x), one
# bench process per run; prints img/s, the per-family ms of the profile pass and the parity figure.
set -o pipefail
ARGS=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for spec in "$@"; do
    envs=""; [ "$spec" != "default" ] && envs="$spec"
    env $envs timeout -k 10 240 python -u bench.py $ARGS --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { echo "bench failed ($spec)"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab.json'))
f=d['roofline']['family_ms_per_forward']
print('[$spec]', '$ARGS', round(d['value']), 'img/s', ' '.join(f'{k}={v:.3f}' for k,v in f.items()), 'parity', d.get('parity',{}).get('max_rel_logit_err_vs_cpu_fp32_oracle'), flush=True)"
  done
done
