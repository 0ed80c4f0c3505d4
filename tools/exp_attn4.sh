#!/bin/bash
# attention_v3 with 64 queries per wave (CLIPVIT_ATTN_V3=3) against 32 (=1): parity, then in-model.
set -o pipefail
mkdir -p gpurun_out
CLIPVIT_ATTN_V3=3 timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/attn4_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|assert|Error" gpurun_out/attn4_tests.log | head; tail -5 gpurun_out/attn4_tests.log; exit 1; }
tail -1 gpurun_out/attn4_tests.log
for M in "ViT-L/14@336px 128 16" "ViT-B/16 256 8"; do set -- $M
  for E in 1 3 1 3; do
    CLIPVIT_ATTN_V3=$E timeout -k 10 200 python -u bench.py --no-cpu-baseline --model $1 --batch $2 --lora-rank $3 --steps 10 --warmup 3 > gpurun_out/attn4.log 2>&1 || { tail gpurun_out/attn4.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/attn4.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('$1 v3=$E', d['value'], d['ms_per_step'], 'attention', round(f['attention'],4))"
  done
done
