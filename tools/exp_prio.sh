#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "86 or 87 or 88 or identity" > gpurun_out/prio_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|assert" gpurun_out/prio_tests.log | head; tail -5 gpurun_out/prio_tests.log; exit 1; }
tail -1 gpurun_out/prio_tests.log
timeout -k 10 120 python -u tools/gemm_tune.py --variants 280,286,213,287 --iters 30 > gpurun_out/prio_a.log 2>&1 || { tail gpurun_out/prio_a.log; exit 1; }
grep -E "qkv|fc" gpurun_out/prio_a.log
timeout -k 10 120 python -u tools/gemm_tune.py --variants 282,288 --epi 0 --iters 30 > gpurun_out/prio_b.log 2>&1 || { tail gpurun_out/prio_b.log; exit 1; }
grep -E "out|proj" gpurun_out/prio_b.log
bash tools/exp_sweep.sh 80,82,13,82,22 86,88,87,88,22
