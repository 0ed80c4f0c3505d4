#!/bin/bash
# r05: MX-fp8 tile costs by epilogue (store16 vs QuickGELU + quantize) against the 16-bit tiles
set -o pipefail
out=gpurun_out/r05_mx_epi
mkdir -p $out
GEMM_AB_DTYPE=3 timeout -k 10 300 python -u tools/gemm_ab.py "12800,3072,768,0;12800,3072,768,1;12800,2304,768,0;12800,768,3072,0" "3,1,2" 5 20 > $out/mx.log 2>&1 || { echo "mx failed"; tail -5 $out/mx.log; exit 1; }
GEMM_AB_DTYPE=2 timeout -k 10 300 python -u tools/gemm_ab.py "12800,3072,768,0;12800,3072,768,1;12800,2304,768,0;12800,768,3072,0" "62,72,10072" 5 20 > $out/f16.log 2>&1 || { echo "f16 failed"; tail -5 $out/f16.log; exit 1; }
cat $out/mx.log $out/f16.log
