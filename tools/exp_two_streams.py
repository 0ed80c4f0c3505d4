"""Experiment: two batches in flight on two HIP streams (two handles, so two workspaces) vs
one stream — does overlapping one batch's latency-bound tail/head with the next batch's
GEMMs raise images/s? (ViT-B/32 + LoRA r=8, fp16, bs 256 per step.)"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
import torch  # noqa: E402

from interior_amd import config as C  # noqa: E402
from interior_amd.engine import VisionEngine  # noqa: E402
from interior_amd.lora import synthetic_adapters  # noqa: E402
from interior_amd.weights import synthetic_state_dict  # noqa: E402

SEG = [0, 40, 60, 359, 395, 425, 437]


def make(cfg, dev, sd, ad, T):
    e = VisionEngine(cfg, dev, "fp16", max_batch=256)
    e.load_state_dict(sd)
    e.load_lora(ad)
    e.set_text_features(T.numpy(), SEG)
    return e


def main():
    dev = torch.device("cuda", 0)
    cfg = C.VIT_B32
    sd, ad = synthetic_state_dict(cfg, 0), synthetic_adapters(cfg, rank=8)
    T = torch.nn.functional.normalize(torch.randn(437, 512, generator=torch.Generator().manual_seed(1)), dim=-1)
    single = "--single" in sys.argv
    e0 = make(cfg, dev, sd, ad, T)
    engs = [e0, e0 if single else make(cfg, dev, sd, ad, T)]
    px = torch.randn(256, 3, 224, 224, device=dev).clamp_(-1.8, 2.2)
    outs = [engs[i].classify(px) for i in range(2)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    K = 40
    for mode in ("one", "two", "two1", "one", "two", "two1"):
        for _ in range(5):
            engs[0].classify(px, outs[0])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            j = i % 2 if mode != "one" else 0
            e = engs[j] if mode == "two" else engs[0]  # two1: two streams, ONE handle
            with torch.cuda.stream(streams[j]):
                e.classify(px, outs[j])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"{mode} stream(s): {K * 256 / el:.0f} img/s, {el / K * 1e3:.3f} ms/step", flush=True)
    a, b = outs[0].logits.clone(), outs[1].logits.clone()
    print("outputs equal across handles:", torch.equal(a, b))


if __name__ == "__main__":
    main()
