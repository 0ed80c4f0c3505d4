#!/bin/bash
# Round 5: variant 72 (gemm_p32.h) — kernel correctness tests, then interleaved kernel A/B
# against the shipped tiles on the B/32 bs-256 shapes and 4096^3. Output under gpurun_out/r05_p32/.
set -o pipefail
out=gpurun_out/r05_p32
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "72" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u tools/gemm_ab.py "10752,3072,768,1;12800,3072,768,1;12800,2304,768,0;4096,4096,4096,0" \
  "3462,3472,62,72" 5 20 > $out/ab.log 2>&1 || { echo "ab failed"; tail -20 $out/ab.log; exit 1; }
cat $out/ab.log
# in-model: the shipped line against v72 as the c_fc main launch, and also as the QKV tile
bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--tuning split_variants=72,81" \
  "--tuning split_variants=72,81;qkv_variant=72" > $out/inmodel.log 2>&1 || { echo "in-model A/B failed"; tail -20 $out/inmodel.log; exit 1; }
cat $out/inmodel.log
