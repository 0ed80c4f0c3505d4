#!/bin/bash
# Write-through (sc1) GEMM output stores vs plain: kernel tests, then in-model bench A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k gemm -x -q --timeout 120 --timeout-method thread > gpurun_out/sc1_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sc1_tests.log; exit 1; }
tail -2 gpurun_out/sc1_tests.log
for r in 1 2; do
  for V in "8,21,13,21,21" "50,51,52,51,51" "8,51,13,51,21" "50,21,52,21,21"; do
    CLIPVIT_GEMM_VARIANTS=$V timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/sc1_b.log 2>&1 || { echo "bench failed $V"; tail gpurun_out/sc1_b.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/sc1_b.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('$V', d['value'], d['ms_per_step'], {k:round(v,3) for k,v in f.items()})"
  done
done
