#!/bin/bash
# Same-box A/B of environment settings on the bench (GPU box, from the repo root):
#   bash tools/ab_envs.sh "<bench args>" ROUNDS "A=1 B=2" "A=3" ...
# Each argument after ROUNDS is one arm (space-separated VAR=value pairs, "-" = no change); the
# arms alternate ROUNDS times, one bench process per run; prints img/s and the per-family ms.
set -o pipefail
ARGS=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for arm in "$@"; do
    E=""; [ "$arm" != "-" ] && E="$arm"
    env $E timeout -k 10 240 python -u bench.py $ARGS --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { echo "bench failed ($arm)"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab.json'))
f=d['roofline']['family_ms_per_forward']
print('[$arm]', '$ARGS', round(d['value']), 'img/s', ' '.join(f'{k}={v:.3f}' for k,v in f.items()), 'parity', d.get('parity',{}).get('max_rel_logit_err_vs_cpu_fp32_oracle'), flush=True)"
  done
done
