"""GEMM tile-variant sweep on the encoder's shapes (run on the GPU box).

    python tools/gemm_tune.py [--batch 256] [--model ViT-B/32] [--iters 20]
Prints one line per (shape, variant): device ms per launch and TFLOP/s on random operands.
"""
import argparse
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
import torch  # noqa: E402
from interior_amd import _lib  # noqa: E402
from interior_amd.config import get_config  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--model", default="ViT-B/32")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--dtype", type=int, default=2)
    p.add_argument("--variants", default="1,2,3,4")
    p.add_argument("--epi", type=int, default=-1, help="force an epilogue (6 = discard ablation)")
    a = p.parse_args()
    torch.cuda.init()
    cfg = get_config(a.model)
    M, D = a.batch * cfg.tokens, cfg.width
    Kp = (3 * cfg.patch_size ** 2 + 63) // 64 * 64
    shapes = [("patch", a.batch * cfg.grid ** 2, D, Kp, 4), ("qkv", M, 3 * D, D, 0),
              ("out", M, D, D, 2), ("fc", M, 4 * D, D, 1), ("proj", M, D, 4 * D, 2)]
    L = _lib.lib()
    for name, m, n, k, epi in shapes:
        epi = epi if a.epi < 0 else a.epi
        for v in map(int, a.variants.split(",")):
            ms = ctypes.c_float()
            rc = L.clipvit_gemm_bench(a.dtype, m, n, k, epi, v, a.iters, ctypes.byref(ms))
            if rc:
                print(f"{name:6s} M={m} N={n} K={k} v{v}: unsupported")
                continue
            tf = 2.0 * m * n * k / (ms.value * 1e-3) / 1e12
            print(f"{name:6s} M={m} N={n} K={k} v{v}: {ms.value * 1e3:8.1f} us  {tf:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
