#!/bin/bash
# Round 5 closing A/B of the shipped defaults against the r04 GEMM defaults, per config.
set -o pipefail
out=gpurun_out/r05_final_ab
mkdir -p $out
OLD="--tuning w_blocked=0;split_variants=62,81;large_variants=3462,3463,3463,3463"
bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "$OLD" > $out/b32.log 2>&1 || { echo "b32 A/B failed"; tail -5 $out/b32.log; exit 1; }
bash tools/ab_envs.sh "--model ViT-B/16 --steps 10 --warmup 3" 2 - "$OLD" > $out/b16.log 2>&1 || { echo "b16 A/B failed"; exit 1; }
bash tools/ab_envs.sh "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2" 2 - "$OLD" > $out/l14.log 2>&1 || { echo "l14 A/B failed"; exit 1; }
cat $out/b32.log $out/b16.log $out/l14.log | cut -c1-120
