#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/auto_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|assert|Error" gpurun_out/auto_tests.log | head; exit 1; }
tail -1 gpurun_out/auto_tests.log
run() {  # label, env, bench args
  env $2 timeout -k 10 200 python -u bench.py --no-cpu-baseline $3 > gpurun_out/auto_b.log 2>&1 || { echo "bench failed $1"; tail gpurun_out/auto_b.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/auto_b.log').read().strip().splitlines()[-1]); f=d['roofline']['family_ms_per_forward']
print('$1', d['value'], d['ms_per_step'], {k:round(v,3) for k,v in f.items()})"
}
run "L14-auto" "X=1" "--model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 4 --warmup 2 --profile-iters 1"
run "B16-auto" "X=1" "--model ViT-B/16 --steps 8 --warmup 2"
run "B16-old" "CLIPVIT_GEMM_VARIANTS=80,82,13,82,22" "--model ViT-B/16 --steps 8 --warmup 2"
run "B16-all80" "CLIPVIT_GEMM_VARIANTS=80,80,80,80,22" "--model ViT-B/16 --steps 8 --warmup 2"
run "B32-auto" "X=1" "--steps 20"
