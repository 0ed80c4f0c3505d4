"""Yardstick: the same ViT-B/32 classify step written in plain PyTorch-ROCm on the GPU (fp16,
hipBLASLt GEMMs, torch SDPA attention, torch LayerNorm; torch.compile is not used), timed like
bench.py. Not part of the product and not an oracle: it only shows what the framework the
reference would run on an MI355X reaches on the same workload.

    python tools/torch_gpu_ref.py [--batch 256] [--steps 20]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
from interior_amd import config as C  # noqa: E402
from interior_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="ViT-B/32")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    a = p.parse_args()
    cfg = C.get_config(a.model)
    dt, dev = torch.float16, "cuda"
    sd = {k: v.to(dev, dt) for k, v in synthetic_state_dict(cfg, 0).items()}
    D, H, P = cfg.width, cfg.heads, cfg.patch_size
    T = F.normalize(torch.randn(437, cfg.embed_dim, device=dev), dim=-1).to(dt)
    px = torch.randn(a.batch, 3, cfg.image_size, cfg.image_size, device=dev).clamp_(-1.8, 2.2).to(dt)
    pre = "visual."

    @torch.no_grad()
    def step(x):
        B = x.shape[0]
        x = F.conv2d(x, sd[pre + "conv1.weight"], stride=P).flatten(2).transpose(1, 2)
        x = torch.cat([sd[pre + "class_embedding"].expand(B, 1, D), x], 1) + sd[pre + "positional_embedding"]
        x = F.layer_norm(x, (D,), sd[pre + "ln_pre.weight"], sd[pre + "ln_pre.bias"])
        N = x.shape[1]
        for i in range(cfg.layers):
            r = f"{pre}transformer.resblocks.{i}."
            h = F.layer_norm(x, (D,), sd[r + "ln_1.weight"], sd[r + "ln_1.bias"])
            qkv = F.linear(h, sd[r + "attn.in_proj_weight"], sd[r + "attn.in_proj_bias"])
            q, k, v = qkv.view(B, N, 3, H, D // H).permute(2, 0, 3, 1, 4)
            o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, N, D)
            x = x + F.linear(o, sd[r + "attn.out_proj.weight"], sd[r + "attn.out_proj.bias"])
            h = F.layer_norm(x, (D,), sd[r + "ln_2.weight"], sd[r + "ln_2.bias"])
            u = F.linear(h, sd[r + "mlp.c_fc.weight"], sd[r + "mlp.c_fc.bias"])
            u = u * torch.sigmoid(1.702 * u)
            x = x + F.linear(u, sd[r + "mlp.c_proj.weight"], sd[r + "mlp.c_proj.bias"])
        f = F.layer_norm(x[:, 0], (D,), sd[pre + "ln_post.weight"], sd[pre + "ln_post.bias"]) @ sd[pre + "proj"]
        f = F.normalize(f.float(), dim=-1)
        return (100.0 * f @ T.float().t()).softmax(-1)

    for _ in range(a.warmup):
        step(px)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(px)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"yardstick": "PyTorch-ROCm eager fp16 (hipBLASLt GEMMs, SDPA)", "model": a.model,
                      "batch": a.batch, "img_per_s": round(a.batch * a.steps / el, 1),
                      "ms_per_step": round(el / a.steps * 1e3, 3), "torch": torch.__version__}))


if __name__ == "__main__":
    main()
