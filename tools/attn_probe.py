"""Attention kernel timing. Default: N = 50 (ViT-B/32) against batch size and against a plain
device copy of the same bytes (bandwidth- or latency-bound?). With arguments "B,N,H" ...: those
shapes only (e.g. 64,577,16 for a ViT-L/14@336 lane, 128,197,12 for ViT-B/16).

    python tools/attn_probe.py [B,N,H ...]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
from interior_amd import engine as E  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


dev = torch.device("cuda", 0)
if len(sys.argv) > 1:
    for arg in sys.argv[1:]:
        B, N, H = map(int, arg.split(","))
        qkv = torch.randn(B * N, 3 * H * 64, device=dev).half()
        t = timeit(lambda: E.attention_test(qkv, B, N, H), iters=20)
        print(f"B={B} N={N} H={H}: attention {t:8.1f} us, {4 * B * H * N * N * 64 / t / 1e6:7.1f} TFLOP/s", flush=True)
    sys.exit(0)
H, N = 12, 50
for B in (32, 64, 128, 256, 512):
    qkv = torch.randn(B * N, 3 * H * 64, device=dev).half()
    t = timeit(lambda: E.attention_test(qkv, B, N, H))
    mb = (qkv.numel() * 2 + B * N * H * 64 * 2) / 1e6
    dst = torch.empty_like(qkv)
    tc = timeit(lambda: dst.copy_(qkv))
    mbc = 2 * qkv.numel() * 2 / 1e6
    print(f"B={B:4d}: attention {t:7.1f} us, {mb:6.1f} MB -> {mb / t:5.2f} TB/s | copy {tc:7.1f} us, "
          f"{mbc:6.1f} MB -> {mbc / tc:5.2f} TB/s", flush=True)
