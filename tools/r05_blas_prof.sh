#!/bin/bash
# r05: which hipBLASLt kernels (macro tile, depth) run the B/32 shapes
set -o pipefail
out=$PWD/gpurun_out/r05_blas_prof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/blas_yardstick.py --dtypes float16 --iters 20 > $out/log.txt 2>&1 || { echo "prof failed"; tail -5 $out/log.txt; exit 1; }
find $out/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-400
