#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
C=""
for shape in "12800,2304,768" "4096,4096,4096"; do
  for v in 8 63 64 62; do C="$C;$shape,6,$v"; done
  for v in 70 72 73 74; do C="$C;$shape,6,$v"; done
done
C=${C#;}
timeout -k 10 200 python -u tools/gemm_multi.py "$C" 30 > gpurun_out/abl3_timing.txt 2>&1 || { echo "timing failed"; tail gpurun_out/abl3_timing.txt; exit 1; }
cat gpurun_out/abl3_timing.txt
