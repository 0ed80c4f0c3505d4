#!/bin/bash
# r06 session 2: store-policy A/Bs beyond the default B/32 line (config 5, bs 128, B/16, L/14@336)
# and the XCD maps of QKV / c_fc once the GEMM outputs no longer stay in L2. Library variants
# from tools/build_alt.py (ppmx17: ping-pong + MX tiles store sc0 sc1; nt17: the large-M c_fc
# (variant 74) stores sc0 sc1 instead of nt).
set -o pipefail
O=gpurun_out/c15
mkdir -p $O
bash tools/ab_envs.sh "--dtype mxfp8 --batch 512 --steps 10 --warmup 3" 3 - "CLIPVIT_LIB=$PWD/alt/ppmx17.so" > $O/ab_cfg5.log 2>&1 && \
bash tools/ab_envs.sh "--batch 128 --steps 20 --warmup 5" 2 - "CLIPVIT_LIB=$PWD/alt/ppmx17.so" > $O/ab_bs128.log 2>&1 && \
bash tools/ab_envs.sh "--model ViT-B/16 --steps 10 --warmup 3" 2 - "CLIPVIT_LIB=$PWD/alt/nt17.so" > $O/ab_b16.log 2>&1 && \
bash tools/ab_envs.sh "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 4 --warmup 2" 2 - "CLIPVIT_LIB=$PWD/alt/nt17.so" > $O/ab_l14.log 2>&1 && \
bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--tuning split_xcd=36" "--tuning split_xcd=38" "--tuning split_xcd=0" "--tuning gemm_xcd=35,0,2,0,1" "--tuning gemm_xcd=41,0,2,0,1" > $O/ab_xcd.log 2>&1
cat $O/*.log
