#!/bin/bash
# r04 second session: full GPU test suite, default bench, headline rocprof round (tag r04b) and
# the config-5 rocprof passes on the final build. Every GPU step under its own time limit; the
# first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
bash tools/profile_round.sh gpurun_out/prof r04b > gpurun_out/prof_round.log 2>&1 || { echo "profile round failed"; tail -20 gpurun_out/prof_round.log; exit 1; }
echo prof-ok
bash tools/profile_cfg5.sh gpurun_out/cfg5prof3 r04b > gpurun_out/cfg5prof3.log 2>&1 || { echo "cfg5 profile failed"; tail -20 gpurun_out/cfg5prof3.log; exit 1; }
echo cfg5-prof-ok
