"""Worker body for tests/test_dp.py (importable in spawned children: registers the package)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
import amd_pkg  # noqa: E402

amd_pkg.load()
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from interior_amd import dp  # noqa: E402


class FakeEngine:
    """Stands in for VisionEngine on CPU: deterministic per-image logits."""

    class Out:
        def __init__(self, logits):
            self.logits = logits

    def classify(self, px, out=None):
        return self.Out(px.reshape(px.shape[0], -1)[:, :5].sum(1, keepdim=True) * torch.arange(1., 8.))


def worker(rank, world, port, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        full = torch.randn(B, 3, 4, 4, generator=g)
        a, b = dp.shard_bounds(B, world, rank)
        logits, _ = dp.ShardedClassifier(FakeEngine()).classify_global(full[a:b], B)
        ok = torch.equal(logits, FakeEngine().classify(full).logits)
        eq = dp.allgather_rows(torch.full((3, 2), float(rank)))
        ok &= torch.equal(eq, torch.cat([torch.full((3, 2), float(r)) for r in range(world)]))
        q.put((rank, bool(ok)))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def gpu_worker(rank, world, port, B, q):
    """config 3's code path on the HIP engine: every rank on cuda:0 (a 1-GPU box), gloo for the
    gather; rank 0 also classifies the whole batch in one call and compares bit for bit."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from interior_amd import config as C
        from interior_amd.engine import VisionEngine
        from interior_amd.lora import synthetic_adapters
        from interior_amd.weights import synthetic_state_dict
        cfg = C.VIT_B32
        dev = torch.device("cuda", 0)
        eng = VisionEngine(cfg, dev, "fp16", max_batch=B)
        eng.load_state_dict(synthetic_state_dict(cfg, 0))
        eng.load_lora(synthetic_adapters(cfg, rank=8))
        g = torch.Generator().manual_seed(5)
        T = torch.nn.functional.normalize(torch.randn(437, cfg.embed_dim, generator=g), dim=-1)
        eng.set_text_features(T.numpy(), [0, 40, 60, 359, 395, 425, 437])
        full = torch.randn(B, 3, 224, 224, generator=g).clamp_(-1.8, 2.2)
        a, b = dp.shard_bounds(B, world, rank)
        logits, res = dp.ShardedClassifier(eng).classify_global(full[a:b].to(dev), B)
        torch.cuda.synchronize()
        ok = tuple(logits.shape) == (B, 437)
        if rank == 0:
            one = eng.classify(full.to(dev))
            torch.cuda.synchronize()
            ok = ok and torch.equal(logits.cpu(), one.logits.cpu()) and \
                torch.equal(res.top_idx.cpu(), one.top_idx[a:b].cpu())
        eng.close()
        q.put((rank, bool(ok)))
    except Exception as e:
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()
