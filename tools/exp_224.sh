#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "83 or 84 or 85 or identity" > gpurun_out/t224.log 2>&1 || { echo "tests failed"; grep -E "FAIL|assert" gpurun_out/t224.log | head; tail -5 gpurun_out/t224.log; exit 1; }
tail -1 gpurun_out/t224.log
for r in 1 2; do
timeout -k 10 120 python -u tools/gemm_tune.py --variants 213,283,284,285,280 --iters 30 > gpurun_out/t224a.log 2>&1 || { tail gpurun_out/t224a.log; exit 1; }
grep -E "qkv|fc" gpurun_out/t224a.log
done
bash tools/exp_sweep.sh 80,82,13,82,22 80,82,283,82,22 80,82,285,82,22
