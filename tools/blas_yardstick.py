"""Vendor-library yardstick for the B/32 bs-256 GEMM shapes (GPU box).

    python tools/blas_yardstick.py [--iters 50] [--out profiles/r05/blas_yardstick.jsonl]

Times torch.nn.functional.linear (hipBLASLt on this image) in fp16 and bf16 (and, with
--dtypes float8_e4m3fn, per-tensor-scaled fp8 torch._scaled_mm against the 5,033 TF/s fp8 peak)
on the encoder's
four Linear shapes at M = 12,800 (ViT-B/32, 256 images x 50 tokens), the c_fc main launch's
10,752 rows, and 4096^3, with HIP events around `iters` back-to-back launches after a warm-up;
prints one JSON line per shape (median of 5 repeats, us per GEMM and TFLOP/s). Bias-free
(the library's epilogue is not the one the encoder fuses): a lower bound on what the vendor
GEMM needs for the MACs and the operand traffic alone. Not part of the product path.
"""
import argparse
import json
import statistics

import torch

SHAPES = [("qkv", 12800, 2304, 768), ("c_fc", 12800, 3072, 768), ("c_fc_main", 10752, 3072, 768),
          ("out_proj", 12800, 768, 768), ("c_proj", 12800, 768, 3072), ("square", 4096, 4096, 4096)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="comma-separated roles (default: all)")
    ap.add_argument("--dtypes", default="float16,bfloat16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lines = []
    for dt in [getattr(torch, t) for t in a.dtypes.split(",")]:
        fp8 = dt == torch.float8_e4m3fn
        for name, M, N, K in SHAPES:
            if a.only and name not in a.only.split(","):
                continue
            g = torch.Generator(device=dev).manual_seed(M + N + K)
            x = torch.randn(M, K, device=dev, generator=g).to(dt)
            w = (torch.randn(N, K, device=dev, generator=g) * (1.0 if fp8 else 0.05)).to(dt)
            if fp8:  # per-tensor scaled fp8 GEMM (hipBLASLt), bf16 out: the MX-fp8 roles' yardstick
                one = torch.ones((), device=dev)
                wt = w.t()
                op = lambda: torch._scaled_mm(x, wt, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)  # noqa: E731
            else:
                op = lambda: torch.nn.functional.linear(x, w)  # noqa: E731
            for _ in range(10):
                op()
            torch.cuda.synchronize()
            reps = []
            for _ in range(5):
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
                for _ in range(a.iters):
                    op()
                t1.record()
                torch.cuda.synchronize()
                reps.append(t0.elapsed_time(t1) * 1e3 / a.iters)
            us = statistics.median(reps)
            tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
            d = {"lib": "torch._scaled_mm (hipBLASLt)" if fp8 else "torch.nn.functional.linear (hipBLASLt)",
                 "dtype": str(dt).split(".")[1], "role": name,
                 "M": M, "N": N, "K": K, "us": round(us, 2), "min_us": round(min(reps), 2),
                 "tflops": round(tf, 1), "frac_of_peak": round(tf / (5033.2 if fp8 else 2516.6), 4)}
            print(json.dumps(d), flush=True)
            lines.append(d)
            del x, w
    if a.out:
        with open(a.out, "w") as f:
            for d in lines:
                f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
