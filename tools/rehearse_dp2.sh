#!/bin/bash
# Two ranks on the one GPU of a gpurun box (--share-gpu: gloo all-gather, a code-path rehearsal
# of the N > 1 bench line, never a scaling point): launcher, env ranks, barrier + max-over-ranks
# timing, the gathered-logits check.
set -o pipefail
mkdir -p gpurun_out/dp2
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --share-gpu --steps 10 --warmup 3 --no-cpu-baseline \
  > gpurun_out/dp2/line.json 2> gpurun_out/dp2/err.log || { echo "dp2 rehearsal failed"; tail -30 gpurun_out/dp2/err.log; exit 1; }
cat gpurun_out/dp2/line.json
