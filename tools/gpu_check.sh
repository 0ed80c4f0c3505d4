#!/bin/bash
# One GPU call: GPU tests, default bench, then (arg "prof") the rocprof passes of
# tools/profile_round.sh. Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -2 gpurun_out/bench.log
if [ "$1" = "prof" ]; then bash tools/profile_round.sh gpurun_out/prof && echo prof-ok; fi
