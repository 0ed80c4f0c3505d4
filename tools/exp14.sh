#!/bin/bash
mkdir -p gpurun_out
for sk in "" "0" "11" "0,11" "0,1,10,11"; do
  echo "skip=$sk" >> gpurun_out/e14.log
  CLIPVIT_MX8_SKIP=$sk timeout -k 10 300 python -m pytest tests/test_gpu_mx8.py -x -q -s -k "config5" 2>&1 | grep "mxfp8 vs" >> gpurun_out/e14.log
done
