#!/bin/bash
# Round 5: blocked weight operand (GemmArgs.blk_w, tuning w_blocked) on the pipelined tiles and
# variant 72 — kernel tests, bit-identity in the model, in-model A/B.
# Output under gpurun_out/r05_w73/.
set -o pipefail
out=gpurun_out/r05_w73
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "gemm and (72 or 100)" > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "blocked_w" > $out/parity.log 2>&1 || { echo "parity failed"; tail -30 $out/parity.log; exit 1; }
tail -2 $out/parity.log
timeout -k 10 300 python -u tools/gemm_ab.py "10752,3072,768,1;2048,3072,768,1;12800,2304,768,0" \
  "3462,3472,13472,81,10081,98,10098" 5 20 > $out/ab.log 2>&1 || { echo "ab failed"; tail -20 $out/ab.log; exit 1; }
cat $out/ab.log
bash tools/ab_envs.sh "--steps 20 --warmup 5" 2 - "--tuning w_blocked=1" \
  "--tuning w_blocked=1;split_variants=72,81" "--tuning w_blocked=1;split_variants=72,81;qkv_variant=3472" \
  > $out/inmodel.log 2>&1 || { echo "in-model A/B failed"; tail -20 $out/inmodel.log; exit 1; }
cat $out/inmodel.log
