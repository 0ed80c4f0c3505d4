"""Interleaved A/B of GEMM tile variants in ONE process (cdna_hip_programming.md §5.4 rule 24).

    python tools/gemm_ab.py "M,N,K,epi;M,N,K,epi" "v1,v2,..." [rounds] [iters]

For every shape, each round times every variant once (clipvit_gemm_bench: `iters` back-to-back
launches on random uniform operands, HIP events), rounds alternate the variant order; prints the
median and min per variant in us and TF/s. epi = internal Epi enum (0 store16, 1 gelu16).
GEMM_AB_DTYPE selects the operand format (1 bf16; 2 fp16, default; 3 MX-fp8, where epi 1 runs
as the MX-fp8 QuickGELU output).
"""
import ctypes
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
from interior_amd import _lib  # noqa: E402

shapes = [tuple(map(int, s.split(","))) for s in sys.argv[1].split(";")]
variants = [int(v) for v in sys.argv[2].split(",")]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
L = _lib.lib()
dtype = int(os.environ.get("GEMM_AB_DTYPE", "2"))
for M, N, K, epi in shapes:
    t = {v: [] for v in variants}
    for r in range(rounds):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            ms = ctypes.c_float()
            if t[v] is not None and L.clipvit_gemm_bench(dtype, M, N, K, epi, v, iters, ctypes.byref(ms)) == 0:
                t[v].append(ms.value * 1e3)
            else:
                t[v] = None
    for v in variants:
        if not t[v]:
            print(f"{M}x{N}x{K} epi{epi} v{v}: unsupported", flush=True)
            continue
        med, mn = statistics.median(t[v]), min(t[v])
        print(f"{M}x{N}x{K} epi{epi} v{v}: median {med:.1f} us ({2 * M * N * K / (med * 1e-6) / 1e12:.0f} TF/s), "
              f"min {mn:.1f} us", flush=True)
