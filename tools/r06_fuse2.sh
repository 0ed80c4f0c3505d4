#!/bin/bash
# r06 session 2: the fused attention sub-block's phases (diagnostic builds: abl1 = no attention
# phase, abl2 = no out_proj k-loop; outputs garbage) and the staggered W_out walk (rot7: workgroup
# b starts at k-step 7 b mod 24), against the default (three kernels) and attn_fuse=1 (the alt builds run fused by default), B/32 bs 256
set -o pipefail
O=gpurun_out/c20
mkdir -p $O
bash tools/ab_envs.sh "--steps 20 --warmup 5 --no-parity" 2 - "--tuning attn_fuse=1" "CLIPVIT_LIB=$PWD/alt/rot7.so" "CLIPVIT_LIB=$PWD/alt/abl1.so" "CLIPVIT_LIB=$PWD/alt/abl2.so" > $O/fuse2_ab.log 2>&1
cat $O/fuse2_ab.log
