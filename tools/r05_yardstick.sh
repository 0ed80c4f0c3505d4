#!/bin/bash
# r05: hipBLASLt (torch linear) against the library's tiles on the B/32 shapes, same box
set -o pipefail
out=gpurun_out/r05_yardstick
mkdir -p $out
timeout -k 10 300 python -u tools/blas_yardstick.py --out $out/blas.jsonl > $out/blas.log 2>&1 || { echo "blas failed"; tail -5 $out/blas.log; exit 1; }
GEMM_AB_DTYPE=2 timeout -k 10 300 python -u tools/gemm_ab.py "12800,2304,768,0;12800,3072,768,0;10752,3072,768,0;12800,768,768,0;12800,768,3072,0;4096,4096,4096,0" "10098,10062,10072,10082,10008" 5 20 > $out/ours.log 2>&1 || { echo "ours failed"; tail -5 $out/ours.log; exit 1; }
cat $out/blas.log $out/ours.log
