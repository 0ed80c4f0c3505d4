"""bench.py's rank launching on CPU (no GPU work): `--gpus N` outside torchrun starts N ranks
itself and validates rank 0's line; under torchrun a WORLD_SIZE other than --gpus exits non-zero.
The self-launched run itself is tests/test_gpu_bench_dp.py::test_bench_self_launch."""
import importlib.util
import json
import os
import subprocess
import sys
import types
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("world,gpus", [("2", "1"), ("1", "2"), ("8", "4")])
def test_world_size_mismatch_exits_nonzero(world, gpus):
    env = dict(os.environ, WORLD_SIZE=world, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", gpus], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-1000:])
    assert "WORLD_SIZE" in r.stderr and not r.stdout.strip()


def _line(**kw):
    d = {"ranks": 4, "n_gpus": 4, "rccl_world": 4, "backend": "nccl", "gather_ok": True, "value": 1.0}
    d.update(kw)
    return json.dumps(d)


@pytest.mark.parametrize("line,share,rc", [
    (_line(), False, 0),
    (_line(ranks=1, n_gpus=1, rccl_world=1), False, 3),    # a 1-rank line under --gpus 4
    (_line(gather_ok=False), False, 3),
    (_line(backend="gloo"), False, 3),                     # a real run must gather over RCCL
    (_line(n_gpus=1, backend="gloo"), True, 0),            # --share-gpu rehearsal: gloo, one device
])
def test_launch_ranks_checks_the_line(monkeypatch, capsys, line, share, rc):
    b = _bench()
    seen = {}

    def fake_run(cmd, env=None, stdout=None, text=None):
        seen["cmd"], seen["env"] = cmd, env
        return types.SimpleNamespace(returncode=0, stdout="noise\n" + line + "\n")

    monkeypatch.setattr(b.subprocess, "run", fake_run)
    a = types.SimpleNamespace(gpus=4, share_gpu=share)
    assert b.launch_ranks(a, ["--gpus", "4", "--steps", "3"]) == rc
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and seen["env"]["MASTER_ADDR"] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")
    out = capsys.readouterr().out.strip().splitlines()
    assert out == [line]               # rank 0's line relayed, nothing else on stdout
    assert b.VisionEngine is None      # the launching process never loaded the engine


def test_launch_ranks_propagates_failure(monkeypatch):
    b = _bench()
    monkeypatch.setattr(b.subprocess, "run",
                        lambda *a, **k: types.SimpleNamespace(returncode=1, stdout=""))
    assert b.launch_ranks(types.SimpleNamespace(gpus=2, share_gpu=False), ["--gpus", "2"]) == 1
