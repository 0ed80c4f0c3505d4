#!/bin/bash
# attention_v3 (32 queries per wave): parity (default = v3 for N > 128; mode 2 also N <= 64),
# then in-model A/B against v2 on L/14@336 (config 4), B/16 and B/32.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or classify or prune" > gpurun_out/attn3_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|assert|Error" gpurun_out/attn3_tests.log | head; tail -5 gpurun_out/attn3_tests.log; exit 1; }
tail -1 gpurun_out/attn3_tests.log
CLIPVIT_ATTN_V3=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or classify or prune" > gpurun_out/attn3b_tests.log 2>&1 || { echo "tests (v3=2) failed"; grep -E "FAIL|assert|Error" gpurun_out/attn3b_tests.log | head; tail -5 gpurun_out/attn3b_tests.log; exit 1; }
tail -1 gpurun_out/attn3b_tests.log
for M in "ViT-L/14@336px 128 16" "ViT-B/16 256 8" "ViT-B/32 256 8"; do set -- $M
  for E in 0 1 2; do
    CLIPVIT_ATTN_V3=$E timeout -k 10 200 python -u bench.py --no-cpu-baseline --model $1 --batch $2 --lora-rank $3 --steps 10 --warmup 3 > gpurun_out/attn3.log 2>&1 || { tail gpurun_out/attn3.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/attn3.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('$1 v3=$E', d['value'], d['ms_per_step'], 'attention', round(f['attention'],4))"
  done
done
