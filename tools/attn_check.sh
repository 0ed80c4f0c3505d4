#!/bin/bash
# GPU: full GPU test suite ("quick": attention tests only), then bench lines of B/32, B/16 and L/14@336 (attention family times).
set -o pipefail
mkdir -p gpurun_out
SEL=""; [ "$1" = "quick" ] && SEL="tests/test_gpu_kernels.py -k attention"
[ "$1" = "quick" ] || SEL="tests"
timeout -k 10 700 python -u -m pytest $SEL -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for m in "" "--model ViT-B/16" "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2"; do
  timeout -k 10 300 python -u bench.py $m --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed $m"; tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab.json')); f=d['roofline']['family_ms_per_forward']
print('$m', round(d['value']), 'img/s', ' '.join(f'{k}={v:.3f}' for k,v in f.items()), 'parity', d['parity']['max_rel_logit_err_vs_cpu_fp32_oracle'], flush=True)"
done
