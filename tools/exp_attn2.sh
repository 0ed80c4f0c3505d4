#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or classify or prune" > gpurun_out/attn_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|assert|Error" gpurun_out/attn_tests.log | head; tail -5 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for M in "ViT-L/14@336px 128 16" "ViT-B/16 256 8"; do set -- $M
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --model $1 --batch $2 --lora-rank $3 --steps 5 --warmup 2 > gpurun_out/attn_l14.log 2>&1 || { tail gpurun_out/attn_l14.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/attn_l14.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('$1', d['value'], d['ms_per_step'], d['roofline']['model_mfma_frac'], {k:round(v,3) for k,v in f.items()})"
done
