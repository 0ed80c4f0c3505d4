#!/bin/bash
# c_fc round split with a 256x192 12-wave main launch (69 direct / 89 staged epilogue):
# c_fc N = 3072 -> 16 N-tiles, rows [0, 12288) = 768 tiles = 3 whole rounds, 512-row tail;
# QKV splits too under this main tile (600 tiles = 2 rounds + 88). Default: "8,81".
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "69 or 89 or identity or bit_identical" > gpurun_out/fc192_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/fc192_tests.log; exit 1; }
tail -2 gpurun_out/fc192_tests.log
bash tools/exp_env.sh "CLIPVIT_SPLIT_VARIANTS=8,81" "CLIPVIT_SPLIT_VARIANTS=69,81" "CLIPVIT_SPLIT_VARIANTS=89,81"
