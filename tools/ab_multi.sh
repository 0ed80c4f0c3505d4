#!/bin/bash
# Same-box A/B of several environment settings on one bench command (GPU box, via gpurun):
#   bash tools/ab_multi.sh "<bench args>" ROUNDS "ENV1=a ENV2=b" "ENV1=c" ...
# each setting is a space-separated list of VAR=value pairs ("-" = the defaults); alternates
# the settings ROUNDS times, one bench process per run.
set -o pipefail
ARGS=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for setting in "$@"; do
    envs=(); [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
    env "${envs[@]}" timeout -k 10 240 python -u bench.py $ARGS --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { echo "bench failed ($setting)"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ab.json')); f=d['roofline']['family_ms_per_forward']
print('[$setting]', round(d['value']), 'img/s', ' '.join(f'{k}={v:.3f}' for k,v in f.items()), flush=True)"
  done
done
