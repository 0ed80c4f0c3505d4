"""Run several GEMM (shape, variant) cases back to back in one process (rocprofv3 PMC passes).

    python tools/gemm_multi.py "M,N,K,epi,var;M,N,K,epi,var;..." [iters]
"""
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
from interior_amd import _lib  # noqa: E402

iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
L = _lib.lib()
for case in sys.argv[1].split(";"):
    M, N, K, epi, var = map(int, case.split(","))
    ms = ctypes.c_float()
    _lib.check(L.clipvit_gemm_bench(2, M, N, K, epi, var, iters, ctypes.byref(ms)))
    print(f"{M}x{N}x{K} epi{epi} v{var}: {ms.value * 1e3:.1f} us  {2 * M * N * K / (ms.value * 1e-3) / 1e12:.1f} TF/s",
          flush=True)
