#!/bin/bash
# LDS-staged row-contiguous epilogue (variants 80-82) vs the direct-store tiles (8, 13, 22).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "80 or 81 or 82 or identity" > gpurun_out/staged_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/staged_tests.log; exit 1; }
tail -2 gpurun_out/staged_tests.log
for r in 1 2; do
timeout -k 10 120 python -u tools/gemm_tune.py --variants 208,280,213,281,222,282 --iters 30 > gpurun_out/staged_a.log 2>&1 || { tail gpurun_out/staged_a.log; exit 1; }
grep -E "qkv|fc" gpurun_out/staged_a.log
timeout -k 10 120 python -u tools/gemm_tune.py --variants 222,282,208,280 --epi 0 --iters 30 > gpurun_out/staged_b.log 2>&1 || { tail gpurun_out/staged_b.log; exit 1; }
grep -E "out|proj" gpurun_out/staged_b.log
done
