#!/bin/bash
# attention_v2 (glds ring + transposed V reads) vs attention_kernel, in-model, B/32 and L/14@336.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or classify or prune" > gpurun_out/attn_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|assert|Error" gpurun_out/attn_tests.log | head; tail -5 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
bash tools/exp_env.sh "CLIPVIT_ATTN_V2=0" "CLIPVIT_ATTN_V2=1" || exit 1
for V in 0 1; do
  CLIPVIT_ATTN_V2=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2 > gpurun_out/attn_l14.log 2>&1 || { tail gpurun_out/attn_l14.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/attn_l14.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('L14 v2=$V', d['value'], d['ms_per_step'], {k:round(v,3) for k,v in f.items()})"
done
