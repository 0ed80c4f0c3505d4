#!/bin/bash
# r06 closing check at HEAD: full GPU suite, smoke(), the default bench line
set -o pipefail
O=gpurun_out/close
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
timeout -k 10 400 python -u bench.py > $O/default.json 2> $O/default.err || { echo "bench failed"; tail -20 $O/default.err; exit 1; }
head -c 400 $O/default.json; echo
