#!/bin/bash
set -o pipefail
out=gpurun_out/r05_w4g
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -m gpu -k "race_screen or gemm_shapes" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
GEMM_AB_DTYPE=2 timeout -k 10 400 python -u tools/gemm_ab.py "12800,2304,768,0;12800,3072,768,1;10752,3072,768,1;12800,768,3072,0;4096,4096,4096,0;36864,4096,1024,1" "10072,10076,3476,10062" 5 20 > $out/ab.log 2>&1 || { echo "ab failed"; tail -5 $out/ab.log; exit 1; }
cat $out/ab.log
