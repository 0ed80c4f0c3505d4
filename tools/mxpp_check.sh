#!/bin/bash
# MX-fp8 ping-pong tile: bit-identity tests, standalone A/B of the MX tiles (tools/gemm_ab.py),
# then the config-5 bench A/B of variant sets (tools/mx_ab.sh) when "ab" is given.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx8.py -x -v --timeout 120 --timeout-method thread > gpurun_out/mxpp_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/mxpp_tests.log; exit 1; }
tail -2 gpurun_out/mxpp_tests.log
GEMM_AB_DTYPE=3 timeout -k 10 240 python -u tools/gemm_ab.py "12800,2304,768,0;12800,3072,768,1;12800,768,3072,0;12800,768,768,0" "2,3" 5 20 || exit 1
if [ "$1" = "ab" ]; then bash tools/mx_ab.sh; fi
