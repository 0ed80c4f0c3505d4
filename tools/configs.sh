#!/bin/bash
# Bench lines of the other BASELINE configs (config 4 L/14@336 bs 128 fp16, B/16 bs 256 fp16,
# config 2 in bf16 at bs 256) and the default line
set -o pipefail
mkdir -p gpurun_out/cfg
timeout -k 10 300 python -u bench.py --model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cfg/cfg4.json 2> gpurun_out/cfg/cfg4.err || { echo "cfg4 failed"; tail -5 gpurun_out/cfg/cfg4.err; exit 1; }
timeout -k 10 300 python -u bench.py --model ViT-B/16 --no-cpu-baseline > gpurun_out/cfg/b16.json 2> gpurun_out/cfg/b16.err || { echo "b16 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > gpurun_out/cfg/cfg2_bf16.json 2> gpurun_out/cfg/cfg2_bf16.err || { echo "bf16 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/cfg/default.json 2> gpurun_out/cfg/default.err || { echo "default failed"; exit 1; }
for f in cfg4 b16 cfg2_bf16 default; do python3 -c "
import json; d=json.load(open('gpurun_out/cfg/$f.json')); print('$f', round(d['value']), d['config']['workload'][:40], d['dtype'], d['config']['per_gpu_batch'], 'frac', d['roofline']['frac'], 'model', d['roofline']['model_mfma_frac'], 'parity', d['parity'])"; done
