#!/bin/bash
# In-model GEMM role variants on config 4 (ViT-L/14@336, bs 128, LoRA r=16).
set -o pipefail
mkdir -p gpurun_out
for V in "$@"; do
  CLIPVIT_GEMM_VARIANTS=$V timeout -k 10 200 python -u bench.py --no-cpu-baseline --model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 4 --warmup 2 --profile-iters 1 > gpurun_out/sweep_l14.log 2>&1 || { echo "bench failed $V"; tail gpurun_out/sweep_l14.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/sweep_l14.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('$V', d['value'], d['ms_per_step'], {k:round(v,2) for k,v in f.items()})"
done
