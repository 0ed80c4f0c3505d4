#!/bin/bash
# Same-box A/B of bench arms (GPU box, from the repo root):
#   bash tools/ab_envs.sh "<bench args>" ROUNDS "--tuning split_min=0" "CLIPVIT_LIB=$PWD/ab/x.so" "-" ...
# Each argument after ROUNDS is one arm: extra bench arguments when it starts with "--" (e.g.
# --tuning "key=value;..." = clipvit_set_tuning), else space-separated VAR=value environment pairs
# (CLIPVIT_LIB: another library build); "-" = no change. The arms alternate ROUNDS times, one
# bench process per run; prints img/s and the per-family ms.
set -o pipefail
ARGS=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for arm in "$@"; do
    E=""; X=()
    case "$arm" in -) ;; --*) X=($arm) ;; *) E="$arm" ;; esac
    env $E timeout -k 10 240 python -u bench.py $ARGS "${X[@]}" --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { echo "bench failed ($arm)"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab.json'))
f=d['roofline']['family_ms_per_forward']
print('[$arm]', '$ARGS', round(d['value']), 'img/s', ' '.join(f'{k}={v:.3f}' for k,v in f.items()), 'parity', d.get('parity',{}).get('max_rel_logit_err_vs_cpu_fp32_oracle'), flush=True)"
  done
done
