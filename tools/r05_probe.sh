#!/bin/bash
# Round-5 GEMM timeline probe (tools/probes/gemm_probe.hip): barrier / MFMA-segment micro-probe,
# then the stamped persistent ping-pong on the B/32 bs-256 shapes. Output under gpurun_out/.
set -o pipefail
out=gpurun_out/r05_probe
mkdir -p $out
P=tools/probes/gemm_probe
run() { echo "== $*"; timeout -k 10 120 $P "$@"; }
{
run bar && \
run 10752 3072 768 1 34 && \
run 12800 2304 768 0 0
} > $out/probe2.txt 2>&1 || { echo "probe failed"; tail -30 $out/probe2.txt; exit 1; }
head -12 $out/probe2.txt
