"""Measurement of the SURVEY.md §8(f) rows beside the headline bench (run on the GPU box):

* preprocess: clipvit_preprocess on B decoded RGB images (640x480 -> 224, the common photo
  shape) — images/s from HIP events on the launch stream, HBM roofline on the algorithmic
  bytes (source RGB read + intermediate rows + fp32 output), vs PIL `_transform` on host
  threads (the reference's CPU path, main.py:436-438);
* text tower: clipvit_encode_text on the reference's 437 prompts (77 tokens) — prompts/s and
  MFMA fraction on the algorithmic FLOPs, vs the oracle's torch-CPU encode_text.

Prints one JSON line per row.
"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import amd_pkg  # noqa: E402

amd_pkg.load()
import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from interior_amd import config as C  # noqa: E402
from interior_amd import labels as L  # noqa: E402
from interior_amd import preprocess as PP  # noqa: E402
from interior_amd import tokenizer as TK  # noqa: E402
from interior_amd.text import TextEngine  # noqa: E402
from interior_amd.weights import synthetic_text_state_dict  # noqa: E402
from oracle import clip_ref  # noqa: E402

PEAK_HBM = 8000.0   # GB/s (MI355X_MICROARCH.md)
PEAK_F16 = 2516.6   # TFLOP/s dense
ROOT = Path(__file__).resolve().parents[1]


def gpu_time(fn, iters):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters  # ms


def row_preprocess(B=256, W=640, H=480, n=224):
    rng = np.random.default_rng(0)
    imgs = [Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8), "RGB") for _ in range(B)]
    dev = torch.device("cuda", 0)
    out = torch.empty((B, 3, n, n), device=dev)
    # stage the RGB bytes once (host decode + PCIe are outside the kernel measurement)
    import ctypes
    from interior_amd import _lib
    arrs = [np.asarray(im) for im in imgs]
    table = (_lib.Image * B)()
    off = 0
    for i, a in enumerate(arrs):
        table[i].offset, table[i].height, table[i].width = off, a.shape[0], a.shape[1]
        off += a.nbytes
    rgb = torch.from_numpy(np.concatenate([a.reshape(-1) for a in arrs])).to(dev)
    Lb = _lib.lib()

    def run():
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(Lb.clipvit_preprocess(s, ctypes.c_void_p(rgb.data_ptr()), table, B, n, _lib.F32,
                                         ctypes.c_void_p(out.data_ptr())))
    ms = gpu_time(run, 20)
    ref = torch.stack([torch.from_numpy(PP.to_pixels(im, n)) for im in imgs[:8]])
    assert torch.equal(out[:8].cpu(), ref), "GPU preprocess differs from PIL"
    # algorithmic bytes: source RGB + the [H, n, 3] uint8 intermediate (written, read) + fp32 output
    per_img = W * H * 3 + H * n * 3 * 2 + 3 * n * n * 4
    gbs = per_img * B / (ms * 1e-3) / 1e9
    # CPU: PIL on host threads, ~5 s
    workers = min(16, os.cpu_count() or 1)
    t0, cnt = time.perf_counter(), 0
    while time.perf_counter() - t0 < 5.0:
        PP.preprocess_batch(imgs[:64], n, workers=workers, pin=False)
        cnt += 64
    cpu = cnt / (time.perf_counter() - t0)
    return {"row": "preprocess (clipvit_preprocess, Pillow-exact bicubic 640x480 -> 224 + crop + normalise)",
            "value": round(B / (ms * 1e-3), 1), "unit": "images/s", "batch": B, "ms_per_batch": round(ms, 4),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM, "unit": "GB/s",
                         "frac": round(gbs / PEAK_HBM, 4), "bytes_per_image": per_img},
            "cpu_baseline": {"value": round(cpu, 1), "unit": "images/s", "cores": workers, "kind": "reference",
                             "sample": f"PIL resize/crop/normalise (preprocess.to_pixels) of {cnt} 640x480 images, ~5 s"},
            "parity": "fp32 output bit-identical to PIL path (checked on 8 images)"}


def row_text(golden=ROOT / "tests" / "golden"):
    cats = L.extract_categories(L.load_training_data(golden / "interior_dataset.json"))
    prompts = L.build_label_table(cats).all_texts
    tok = TK.SimpleTokenizer(TK.learn_merges(prompts, 600))
    tc = C.TextConfig(512, 12, 8, 77, tok.vocab_size, 512)
    sd = synthetic_text_state_dict(tc, 1)
    ids = tok.tokenize(prompts)
    B = ids.shape[0]
    eng = TextEngine(tc, 0, "fp16", max_batch=B)
    eng.load_state_dict(sd)
    dev_ids = torch.from_numpy(ids).cuda()
    out = torch.empty((B, 512), device="cuda")
    import ctypes
    from interior_amd import _lib

    def run():
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(_lib.lib().clipvit_encode_text(eng._h, s, ctypes.c_void_p(dev_ids.data_ptr()), B, 1,
                                                  ctypes.c_void_p(out.data_ptr())))
    ms = gpu_time(run, 20)
    ref = torch.nn.functional.normalize(clip_ref.encode_text(sd, ids[:16]), dim=-1)
    err = float((out[:16].cpu() - ref).abs().max())
    tf = B * tc.gflop_per_text() / (ms * 1e-3) / 1e3
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    t0, cnt = time.perf_counter(), 0
    while time.perf_counter() - t0 < 5.0:
        clip_ref.encode_text(sd, ids[:32])
        cnt += 32
    cpu = cnt / (time.perf_counter() - t0)
    eng.close()
    return {"row": "text tower (clipvit_encode_text, 12 x 512 causal, 77 tokens, the reference's 437 prompts)",
            "value": round(B / (ms * 1e-3), 1), "unit": "prompts/s", "batch": B, "ms_per_batch": round(ms, 4),
            "roofline": {"bound": "mfma", "achieved": round(tf, 1), "peak": PEAK_F16, "unit": "TFLOP/s",
                         "frac": round(tf / PEAK_F16, 4), "gflop_per_prompt": round(tc.gflop_per_text(), 4)},
            "cpu_baseline": {"value": round(cpu, 1), "unit": "prompts/s", "cores": torch.get_num_threads(),
                             "kind": "port", "sample": f"oracle encode_text, {cnt} prompts in batches of 32, ~5 s"},
            "parity": f"max |normalised feature diff| vs oracle {err:.2e} (16 prompts)"}


if __name__ == "__main__":
    torch.cuda.init()
    for f in (row_preprocess, row_text):
        print(json.dumps(f()), flush=True)
