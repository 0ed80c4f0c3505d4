#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k gemm -x -q --timeout 120 --timeout-method thread > gpurun_out/deep_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/deep_tests.log; exit 1; }
tail -2 gpurun_out/deep_tests.log
C=""
for v in 208 70 71 270; do C="$C;12800,2304,768,0,$v;12800,2304,768,6,$v"; done
for v in 221 70 71 270; do C="$C;12800,768,768,2,$v"; done
for v in 213 8 70 71 270; do C="$C;12800,3072,768,1,$v"; done
for v in 221 70 71 270; do C="$C;12800,768,3072,2,$v"; done
for v in 8 70 71; do C="$C;4096,4096,4096,0,$v"; done
C=${C#;}
timeout -k 10 200 python -u tools/gemm_multi.py "$C" 30 > gpurun_out/deep_timing.txt 2>&1 || { echo "timing failed"; tail gpurun_out/deep_timing.txt; exit 1; }
cat gpurun_out/deep_timing.txt
