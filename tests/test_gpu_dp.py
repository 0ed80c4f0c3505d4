"""BASELINE config 3's code path (whole-image DP + all-gather of per-image logits) on the HIP
engine: 2 ranks share cuda:0 of the 1-GPU test box (gloo carries the gather; RCCL refuses two
ranks on one device), the gathered [B, 437] logits must equal a 1-rank classify of the full
batch BIT FOR BIT (images are independent: SURVEY.md §8(e), main.py:440-448), ragged B too.
B = 512 is config 3's per-rank workload: 256 ViT-B/32 + LoRA r=8 images per rank (fp16, the
benched dtype), gathered into [512, 437] logits."""
import pytest
import torch.multiprocessing as mp

from test_dp import _free_port

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B", [16, 13, 512])
def test_two_ranks_gather_equals_one_rank_bitwise(gpu, B):
    import _dp_worker
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker.gpu_worker, args=(r, 2, port, B, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert res == {0: True, 1: True}, res
