#!/bin/bash
# Config 5 ratio on one box: bf16 bs 512 and MX-fp8 bs 512 bench lines, alternating ROUNDS times
# (default 2); the JSON lines go to gpurun_out/cfg5_ratio_{bf16,mxfp8}_<round>.json.
set -o pipefail
R=${1:-2}
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for dt in bf16 mxfp8; do
    timeout -k 10 300 python -u bench.py --dtype $dt --batch 512 > gpurun_out/cfg5_ratio_${dt}_$r.json 2> gpurun_out/cfg5_ratio.err \
      || { echo "bench failed ($dt)"; tail -5 gpurun_out/cfg5_ratio.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/cfg5_ratio_${dt}_$r.json')); print('$dt', round(d['value']), 'img/s', d.get('parity'))"
  done
done
