#!/bin/bash
# Closing check at HEAD: full GPU test suite, the default bench line and the config-5 pair
# (MX-fp8 and bf16 at bs 512). Every GPU step under its own time limit; the first failure ends
# the call.
set -o pipefail
mkdir -p gpurun_out/confirm
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/confirm/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/confirm/gpu_tests.log; exit 1; }
tail -2 gpurun_out/confirm/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/confirm/default.json 2> gpurun_out/confirm/default.err \
  || { echo "bench failed"; tail -20 gpurun_out/confirm/default.err; exit 1; }
cat gpurun_out/confirm/default.json
timeout -k 10 400 python -u bench.py --dtype mxfp8 --batch 512 > gpurun_out/confirm/cfg5_mx.json 2> gpurun_out/confirm/cfg5_mx.err \
  || { echo "cfg5 mx bench failed"; tail -20 gpurun_out/confirm/cfg5_mx.err; exit 1; }
cat gpurun_out/confirm/cfg5_mx.json
timeout -k 10 400 python -u bench.py --dtype bf16 --batch 512 > gpurun_out/confirm/cfg5_bf16.json 2> gpurun_out/confirm/cfg5_bf16.err \
  || { echo "cfg5 bf16 bench failed"; tail -20 gpurun_out/confirm/cfg5_bf16.err; exit 1; }
cat gpurun_out/confirm/cfg5_bf16.json
