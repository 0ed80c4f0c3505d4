#!/bin/bash
# r06 session 2: the fused attention sub-block with the out_proj k-steps interleaved with the head pairs: its engine test, then
# the in-model A/B against the three kernels (default) with tuning attn_fuse=1, B/32 bs 256
set -o pipefail
O=gpurun_out/c22
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -s -k "fusion" --timeout 300 --timeout-method thread > $O/fuse_tests.log 2>&1 || { echo "fusion tests failed"; tail -40 $O/fuse_tests.log; exit 1; }
tail -2 $O/fuse_tests.log
bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "--tuning attn_fuse=1" > $O/fuse_ab.log 2>&1
cat $O/fuse_ab.log
