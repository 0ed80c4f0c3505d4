#!/bin/bash
# r06 session 2: config 5 (MX-fp8 bs 512, two lanes) store policy of the MX tiles' MX-fp8 outputs
# (mxq17: the c_fc QuickGELU + quantize epilogue stores sc0 sc1; 16-bit outputs stay plain) and
# the 32x32x64 MX tile (variant 4) on c_fc, against the bf16 bs-512 line of the same box
set -o pipefail
O=gpurun_out/c18
mkdir -p $O
bash tools/ab_envs.sh "--dtype mxfp8 --batch 512 --steps 10 --warmup 3" 3 - "CLIPVIT_LIB=$PWD/alt/mxq17.so" "--tuning mx8_variants=3,5,4,3" > $O/mx_ab.log 2>&1
bash tools/ab_envs.sh "--dtype bf16 --batch 512 --steps 10 --warmup 3" 2 - > $O/bf16_512.log 2>&1
cat $O/mx_ab.log $O/bf16_512.log
