#!/bin/bash
# Round 5: variant 72 operand layout / k-rotation experiments on c_fc main and QKV
# (tools/probes/gemm_probe p32). Output under gpurun_out/r05_p32/.
set -o pipefail
out=gpurun_out/r05_p32
mkdir -p $out
{ echo "== c_fc main 10752x3072x768 gelu xcd34"; timeout -k 10 60 tools/probes/gemm_probe p32 10752 3072 768 1 34 && \
  echo "== QKV 12800x2304x768 xcd0"; timeout -k 10 60 tools/probes/gemm_probe p32 12800 2304 768 0 0; } > $out/layout3.log 2>&1 \
  || { echo "layout probe failed"; tail -20 $out/layout3.log; exit 1; }
grep -v "^  step\|^tile\|epilogue of" $out/layout3.log
