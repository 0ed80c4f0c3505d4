"""Data-parallel path on CPU: 2 ranks over gloo (the GPU run uses the same code over RCCL)."""
import socket

import pytest
import torch.multiprocessing as mp

from interior_amd import dp


def test_shard_bounds_cover_exactly():
    for B in (1, 7, 256, 2048, 2049):
        for W in (1, 2, 3, 8):
            spans = [dp.shard_bounds(B, W, r) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("B", [8, 7])
def test_sharded_classify_gathers_full_batch(B):
    """Each rank classifies its contiguous shard; the all-gather returns the full batch's
    logits in order on every rank, also for ragged shards (B = 7 over 2 ranks)."""
    import _dp_worker
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker.worker, args=(r, 2, port, B, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
