#!/bin/bash
# r06 session 2: the full GPU suite at the current default build, then the store policy of the
# streaming kernels' outputs (ew17: LayerNorm x24 / h and im2col stores sc0 sc1; att17: attention
# output sc0 sc1), B/32 bs 256, same box, 3 alternations
set -o pipefail
O=gpurun_out/c16
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "CLIPVIT_LIB=$PWD/alt/ew17.so" "CLIPVIT_LIB=$PWD/alt/att17.so" > $O/ab_stream.log 2>&1
cat $O/ab_stream.log
