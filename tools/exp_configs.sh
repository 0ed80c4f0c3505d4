#!/bin/bash
# Secondary BASELINE configs + the N-rank bench path rehearsed on one GPU (gloo all-gather).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --no-cpu-baseline --model "ViT-L/14@336px" --batch 128 --lora-rank 16 --steps 5 --warmup 2 > gpurun_out/cfg4.log 2>&1 || { echo "cfg4 failed"; tail gpurun_out/cfg4.log; exit 1; }
tail -1 gpurun_out/cfg4.log | cut -c1-900
timeout -k 10 200 python -u bench.py --no-cpu-baseline --dtype mxfp8 --batch 512 --steps 10 > gpurun_out/cfg5.log 2>&1 || { echo "cfg5 failed"; tail gpurun_out/cfg5.log; exit 1; }
tail -1 gpurun_out/cfg5.log | cut -c1-900
timeout -k 10 200 python -u bench.py --no-cpu-baseline --dtype bf16 --batch 512 --steps 10 > gpurun_out/cfg5b.log 2>&1 || { echo "cfg5b failed"; tail gpurun_out/cfg5b.log; exit 1; }
tail -1 gpurun_out/cfg5b.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --share-gpu --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/dp2.log 2>&1 || { echo "dp2 failed"; tail -20 gpurun_out/dp2.log; exit 1; }
grep metric gpurun_out/dp2.log | cut -c1-400
