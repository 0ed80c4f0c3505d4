"""Run one GEMM shape/variant N times (for rocprofv3 counter passes)."""
import ctypes, sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg; amd_pkg.load()
from interior_amd import _lib
M, N, K, epi, var, iters = map(int, sys.argv[1:7])
ms = ctypes.c_float()
_lib.check(_lib.lib().clipvit_gemm_bench(2, M, N, K, epi, var, iters, ctypes.byref(ms)))
print(f"{M}x{N}x{K} v{var}: {ms.value*1e3:.1f} us  {2*M*N*K/(ms.value*1e-3)/1e12:.1f} TF/s")
