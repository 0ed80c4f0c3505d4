"""Tile variants on the last block's class-token GEMMs (M = batch): out, c_fc, c_proj."""
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
import torch  # noqa: E402
from interior_amd import _lib  # noqa: E402

torch.cuda.init()
L = _lib.lib()
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
vs = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1,4,9,10,11,12,13,22,82").split(",")]
for name, n, k, epi in (("out", 768, 768, 0), ("fc", 3072, 768, 1), ("proj", 768, 3072, 2)):
    for v in vs:
        ms = ctypes.c_float()
        rc = L.clipvit_gemm_bench(2, M, n, k, epi, v, 50, ctypes.byref(ms))
        print(f"{name:5s} M={M} N={n} K={k} v{v}: " + ("unsupported" if rc else f"{ms.value * 1e3:7.1f} us"), flush=True)
