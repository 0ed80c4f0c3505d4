"""One-GPU check of the RCCL calls the DP bench makes (bench.py world > 1): init_process_group
("nccl", device_id=...) and all_gather_into_tensor of the [256, 437] fp32 logits, run as a
world of 1 under torchrun (a 1-GPU box cannot hold two RCCL ranks; the N-rank data path is
covered by tests/test_dp.py over gloo and tests/test_gpu_dp.py).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29531 tools/rccl_check.py
"""
import os
import time

import torch
import torch.distributed as dist

rank, local_rank, world = (int(os.environ.get(k, d)) for k, d in (("RANK", 0), ("LOCAL_RANK", 0), ("WORLD_SIZE", 1)))
dev = torch.device("cuda", local_rank)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x = torch.arange(256 * 437, device=dev, dtype=torch.float32).reshape(256, 437) + rank
out = torch.empty((world * 256, 437), device=dev, dtype=torch.float32)
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
assert torch.equal(out[rank * 256:(rank + 1) * 256], x)
t0 = time.perf_counter()
for _ in range(100):
    dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 100
print(f"rccl all_gather_into_tensor ok: world {world}, backend {dist.get_backend()}, "
      f"{x.numel() * 4 / 1e3:.0f} KB per rank, {dt * 1e6:.1f} us per call", flush=True)
dist.barrier()
dist.destroy_process_group()
