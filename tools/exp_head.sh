#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/head_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/head_tests.log; exit 1; }
tail -2 gpurun_out/head_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/head_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/head_bench.log 2>&1 || { echo "prof failed"; exit 1; }
cd $GRAFT_REPO_ROOT; tail -1 gpurun_out/head_bench.log | cut -c1-300
grep -E "cls_ln|logits_kernel|seg_softmax" gpurun_out/head_prof/run_kernel_stats.csv | cut -c1-150
