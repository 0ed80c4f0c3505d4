#!/bin/bash
# Full GPU test suite, then smoke(): each under its own time limit, the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out/c13
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c13/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/c13/gpu_tests.log; exit 1; }
tail -2 gpurun_out/c13/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
