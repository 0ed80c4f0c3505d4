"""Wave-quantization probe: one GEMM over all M rows vs. a 256x256-tile launch over whole rounds
of tiles followed by a small-tile launch over the remaining rows (run on the GPU box).

    python tools/split_probe.py
"""
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
from interior_amd import _lib  # noqa: E402


def t(M, N, K, epi, var, iters=30):
    ms = ctypes.c_float()
    _lib.check(_lib.lib().clipvit_gemm_bench(2, M, N, K, epi, var, iters, ctypes.byref(ms)))
    return ms.value * 1e3


def main():
    M = 12800
    for name, N, K, epi, full_vars, main_vars, tail_vars, splits in [
        ("fc", 3072, 768, 1, [213, 13, 208, 8, 280], [208, 8, 280], [213, 13, 281, 211, 222], [10752, 11264]),
        ("qkv", 2304, 768, 0, [280, 208, 213], [280, 208], [213, 281, 222, 280], [7168, 9216]),
    ]:
        for v in full_vars:
            us = t(M, N, K, epi, v)
            print(f"{name} full v{v}: {us:.1f} us  {2*M*N*K/us/1e6:.0f} TF/s", flush=True)
        for m1 in splits:
            for vm in main_vars:
                a = t(m1, N, K, epi, vm)
                for vt in tail_vars:
                    b = t(M - m1, N, K, epi, vt)
                    print(f"{name} split {m1}+{M-m1} v{vm}+v{vt}: {a:.1f} + {b:.1f} = {a+b:.1f} us", flush=True)


if __name__ == "__main__":
    main()
