"""Config 5: MX-fp8 logit error against the bf16 engine for several sets of bf16 blocks
(tuning mx8_skip), at the CLIP logit scale of tests/test_gpu_mx8.py (peaked text rows) and on
random text rows; several seeds of images and text.

    python tools/mx_skip_sweep.py "0,1,10,11" "0,10,11" "11|0,1,10,11" ...

An argument "A|M" keeps the attention roles (QKV, out_proj) of blocks A and the MLP roles of
blocks M in bf16 (tuning mx8_skip / mx8_skip_mlp); a plain list sets both.
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
from interior_amd import config as C  # noqa: E402
from interior_amd.engine import VisionEngine  # noqa: E402
from interior_amd.lora import synthetic_adapters  # noqa: E402
from interior_amd.weights import synthetic_state_dict  # noqa: E402

SEGS = [0, 40, 60, 359, 395, 425, 437]


def peaked(anchor, seed, a=0.3):
    g = torch.Generator().manual_seed(seed)
    T = torch.nn.functional.normalize(torch.randn(437, anchor.numel(), generator=g), dim=-1)
    return torch.nn.functional.normalize(a * anchor[None, :] + (1 - a * a) ** 0.5 * T, dim=-1)


def engine(cfg, dtype, sd, ad, B, dev, tuning=None):
    e = VisionEngine(cfg, dev, dtype, max_batch=B, tuning=tuning)
    e.load_state_dict(sd)
    e.load_lora(ad)
    return e


def main():
    dev = torch.device("cuda", 0)
    cfg = C.get_config("ViT-B/32")
    sd = synthetic_state_dict(cfg, 0)
    ad = synthetic_adapters(cfg, rank=8)
    B = 64
    e16 = engine(cfg, "bf16", sd, ad, B, dev)
    cases = []
    for seed in (1234, 77, 92):
        g = torch.Generator().manual_seed(seed)
        px = torch.randn(B, 3, 224, 224, generator=g).clamp_(-1.8, 2.2).to(dev)
        held = torch.randn(8, 3, 224, 224, generator=g).clamp_(-1.8, 2.2).to(dev)
        Tr = torch.nn.functional.normalize(torch.randn(437, cfg.embed_dim, generator=g), dim=-1)
        e16.set_text_features(Tr.numpy(), SEGS)
        f = e16.encode_image(held).cpu()
        anchor = torch.nn.functional.normalize(torch.nn.functional.normalize(f, dim=-1).mean(0), dim=0)
        for name, T in (("peaked", peaked(anchor, seed + 7)), ("random", Tr)):
            e16.set_text_features(T.numpy(), SEGS)
            cases.append((seed, name, px, T, e16.classify(px).logits.cpu()))
    for skip in sys.argv[1:]:
        att, _, mlp = skip.partition("|")
        tun = {"mx8_skip": att}
        if mlp:
            tun["mx8_skip_mlp"] = mlp
        e8 = engine(cfg, "mxfp8", sd, ad, B, dev, tuning=tun)
        res = {"peaked": [], "random": []}
        for seed, name, px, T, ref in cases:
            e8.set_text_features(T.numpy(), SEGS)
            l8 = e8.classify(px).logits.cpu()
            res[name].append(((l8 - ref).abs().amax(1) / ref.abs().amax(1)).max().item())
        e8.close()
        print(f"skip {skip!r:>14}: peaked max {max(res['peaked']):.4g} ({', '.join(f'{v:.4g}' for v in res['peaked'])}); "
              f"random max {max(res['random']):.4g}", flush=True)
    e16.close()


if __name__ == "__main__":
    main()
