#!/bin/bash
# One GPU call: GPU tests, default bench, then (arg "prof") the rocprof passes of
# tools/profile_round.sh. Every GPU step has its own time limit; the first failure ends the call
# (a test failure included: nothing else runs on the GPU after a failed or timed-out step).
set -o pipefail
mkdir -p gpurun_out
if [ "$1" != "nontest" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/gpu_tests.log
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
if [ "$1" = "prof" ] || [ "$2" = "prof" ]; then bash tools/profile_round.sh gpurun_out/prof r03 && echo prof-ok; fi
