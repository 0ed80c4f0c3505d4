#!/bin/bash
# Ablation of the 256x256 pipelined GEMM (v8): where does the time go?
set -o pipefail
mkdir -p gpurun_out
C=""
for shape in "12800,2304,768" "12800,3072,768" "4096,4096,4096"; do
  for e in 0 6; do for v in 8 60 61 62 63 64; do C="$C;$shape,$e,$v"; done; done
done
C=${C#;}
timeout -k 10 200 python -u tools/gemm_multi.py "$C" 30 > gpurun_out/abl_timing.txt 2>&1 || { echo "timing failed"; tail gpurun_out/abl_timing.txt; exit 1; }
cat gpurun_out/abl_timing.txt
