#!/bin/bash
# Round 5: variant 74 (72 with non-temporal stores) for the large-M c_fc — tests, then A/B on
# B/16 and L/14@336 against the shipped 3472 c_fc. Output under gpurun_out/r05_nt/.
set -o pipefail
out=gpurun_out/r05_nt
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread \
  -k "(gemm and 74) or p32_race" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
bash tools/ab_envs.sh "--model ViT-B/16 --steps 10 --warmup 3" 2 - "--tuning large_variants=3462,3474,3463,3463" > $out/b16.log 2>&1 \
  || { echo "b16 A/B failed"; tail -5 $out/b16.log; exit 1; }
bash tools/ab_envs.sh "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2" 2 - "--tuning large_variants=3472,3474,3472,3472" > $out/l14.log 2>&1 \
  || { echo "l14 A/B failed"; tail -5 $out/l14.log; exit 1; }
cat $out/b16.log $out/l14.log | cut -c1-230
