#!/bin/bash
# r06 session 2 final build: rocprof passes of the default bench (tools/profile_round.sh, tag r06c)
# and the other BASELINE configs' lines (tools/profile_configs.sh)
set -o pipefail
bash tools/profile_round.sh gpurun_out/prof r06c || { echo "profile failed"; exit 1; }
bash tools/profile_configs.sh gpurun_out/cfg || { echo "configs failed"; exit 1; }
python3 -c "
import json
for f in ['gpurun_out/prof/bench_traffic.json','gpurun_out/cfg/cfg2_bf16.json','gpurun_out/cfg/cfg2_bf16_bs512.json','gpurun_out/cfg/cfg4.json','gpurun_out/cfg/cfg5.json']:
    d=json.load(open(f)); print(f, round(d['value']), d['dtype'], d['roofline']['frac'], d.get('parity'))
"
