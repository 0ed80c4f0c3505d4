#!/bin/bash
# Bench lines + rocprofv3 kernel statistics of BASELINE.json's other configs (GPU box):
#   config 2 in bf16 (the BASELINE dtype; the line carries its measured parity error),
#   config 4 (ViT-L/14@336 + LoRA r=16, fp16, bs 128), config 5 (MX-fp8 Linears, bs 512).
set -o pipefail
OUT=${1:-gpurun_out/cfg}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py --dtype bf16 --no-cpu-baseline > "$OUT/cfg2_bf16.json" 2> "$OUT/cfg2_bf16.err" || { echo "cfg2 bf16 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --dtype bf16 --batch 512 --no-cpu-baseline > "$OUT/cfg2_bf16_bs512.json" 2> "$OUT/cfg2_bf16_bs512.err" || { echo "cfg2 bf16 bs512 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/cfg4.json" 2> "$OUT/cfg4.err" || { echo "cfg4 failed"; exit 1; }
timeout -k 10 300 python -u bench.py --dtype mxfp8 --batch 512 --no-cpu-baseline > "$OUT/cfg5.json" 2> "$OUT/cfg5.err" || { echo "cfg5 failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/kt4" -o run \
  -- python3 "$ROOT/bench.py" --model ViT-L/14@336px --batch 128 --lora-rank 16 --steps 3 --warmup 1 --no-cpu-baseline --profile-iters 1 > "$ROOT/$OUT/kt4.log" 2>&1 || { echo "cfg4 prof failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/kt5" -o run \
  -- python3 "$ROOT/bench.py" --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline --profile-iters 1 > "$ROOT/$OUT/kt5.log" 2>&1 || { echo "cfg5 prof failed"; exit 1; }
echo configs-done
