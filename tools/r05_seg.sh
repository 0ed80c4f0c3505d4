#!/bin/bash
# Round-5 ping-pong segment-cost micro-probe (tools/probes/gemm_probe bar). Output under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out/r05_probe
timeout -k 10 120 tools/probes/gemm_probe bar > gpurun_out/r05_probe/seg.txt 2>&1 || { tail -20 gpurun_out/r05_probe/seg.txt; exit 1; }
cat gpurun_out/r05_probe/seg.txt
