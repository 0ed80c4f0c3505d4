"""Yardstick: hipBLASLt (torch.matmul) on the encoder's GEMM shapes + a large square GEMM.

    python tools/blas_ref.py [--batch 256]
Not part of the product; prints device us per launch and TFLOP/s.
"""
import argparse

import torch


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--iters", type=int, default=50)
    a = p.parse_args()
    M = a.batch * 50
    shapes = [("qkv", M, 2304, 768), ("out", M, 768, 768), ("fc", M, 3072, 768),
              ("proj", M, 768, 3072), ("sq8192", 8192, 8192, 8192)]
    for dt in (torch.float16, torch.bfloat16):
        for name, m, n, k in shapes:
            A = torch.randn(m, k, device="cuda", dtype=dt)
            W = torch.randn(n, k, device="cuda", dtype=dt)
            for _ in range(5):
                A @ W.t()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                A @ W.t()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            print(f"{str(dt):15s} {name:7s} M={m} N={n} K={k}: {ms * 1e3:8.1f} us "
                  f"{2.0 * m * n * k / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
