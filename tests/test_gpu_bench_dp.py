"""bench.py's multi-rank path (what the driver's N-GPU scaling runs launch) rehearsed on one GPU:
two torchrun ranks share cuda:0 (--share-gpu: gloo, since RCCL refuses two ranks on one device).
Checks the line's contract: the per-rank barrier and max-over-ranks timing ran, the value counts
both ranks' images, and the rehearsal is labelled as such (n_gpus 1, ranks 2, not a scaling
point), and the line reports what the collective did: the world size the process group saw, its
backend, and gather_ok (rank 0's slice of the gathered logits equals its local logits bit for
bit, checked once after the timed loop). On the driver's N-GPU runs the backend is nccl (RCCL);
here it is gloo. The RCCL calls themselves are checked by tools/rccl_check.py."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def test_bench_two_rank_rehearsal(gpu):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29547", str(ROOT / "bench.py"), "--gpus", "2",
           "--share-gpu", "--batch", "32", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--profile-iters", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["ranks"] == 2, d
    assert "not a scaling point" in d["config"]["parallelism"], d["config"]
    assert d["config"]["global_batch"] == 64 and d["steps"] == 3
    assert d["value"] > 0 and abs(d["value"] - 64 * 3 / (d["ms_per_step"] * 3e-3)) / d["value"] < 1e-3
    assert d["parity"]["meets_bar"], d["parity"]
    assert d["rccl_world"] == 2 and d["backend"] == "gloo" and d["gather_ok"] is True, d
    assert d["gathered_rows"] == 64


def test_bench_self_launch(gpu):
    """`python bench.py --gpus 2` with no torchrun: bench.py starts the two ranks itself
    (launch_ranks) and relays rank 0's line, which must report both ranks and a verified gather."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--share-gpu", "--batch", "32",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--profile-iters", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["ranks"] == 2 and d["rccl_world"] == 2 and d["gather_ok"] is True, d
    assert d["config"]["global_batch"] == 64 and d["gathered_rows"] == 64
    assert "launching 2 ranks" in r.stderr
