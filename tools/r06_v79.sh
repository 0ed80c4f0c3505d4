#!/bin/bash
# r06 session 2: variant 79 (the 32-deep-k-step tile at 192 x 256 rows x columns) for the N = 768
# roles: its GEMM tests, kernel-level A/B against v82 (c_proj with blocked u and W: + 30000;
# out_proj with blocked W: + 10000), then in-model B/32 bs 256 arms (same box, 3 alternations)
set -o pipefail
O=gpurun_out/c16
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "79 or race" --timeout 300 --timeout-method thread > $O/v79_tests.log 2>&1 || { echo "v79 tests failed"; tail -30 $O/v79_tests.log; exit 1; }
tail -2 $O/v79_tests.log
timeout -k 10 300 python -u tools/gemm_ab.py "12800,768,3072,0" "30082,30079,30022" 5 20 > $O/v79_kernel.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_ab.py "12800,768,768,0" "10082,10079,10022" 5 20 >> $O/v79_kernel.log 2>&1 || { echo "gemm_ab failed"; cat $O/v79_kernel.log; exit 1; }
cat $O/v79_kernel.log
bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "--tuning proj_variant=79" "--tuning out_variant=79" "--tuning proj_variant=79;out_variant=79" > $O/v79_ab.log 2>&1
cat $O/v79_ab.log
