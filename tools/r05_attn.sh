#!/bin/bash
# Round 5: the persistent attention pair loop (attention_pp_kernel) — kernel tests, attention
# timing, then a same-box A/B against the previous build (ab/base.so). Output gpurun_out/r05_attn/.
set -o pipefail
out=gpurun_out/r05_attn
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  -k "attention_pair" > $out/tests.log 2>&1 || { echo "attention tests failed"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python -u tools/attn_probe.py 256,50,12 > $out/probe_new.log 2>&1 || { echo probe failed; tail -5 $out/probe_new.log; exit 1; }
CLIPVIT_LIB=$PWD/abase/base.so timeout -k 10 120 python -u tools/attn_probe.py 256,50,12 > $out/probe_base.log 2>&1 || { echo probe failed; exit 1; }
echo "new: $(cat $out/probe_new.log | tail -1)"; echo "base: $(cat $out/probe_base.log | tail -1)"
bash tools/ab_envs.sh "--steps 20 --warmup 5" 3 - "CLIPVIT_LIB=$PWD/abase/base.so" > $out/ab.log 2>&1 || { echo "A/B failed"; tail -20 $out/ab.log; exit 1; }
cat $out/ab.log
