#!/bin/bash
# r04 closing session: c_fc tail tiles 64x192 (83, 512 tiles = one 2-per-CU round at bs 256) and
# 128x192 (84, 256 tiles) against the shipped 128x128 (81): GEMM tests of the new tiles, then the
# same-box bench A/B (split_variants main,tail).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "83 or 84 or identity" > gpurun_out/ab9_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/ab9_tests.log; exit 1; }
tail -1 gpurun_out/ab9_tests.log
bash tools/ab_envs.sh "" 2 - "--tuning split_variants=62,83" "--tuning split_variants=62,84"
