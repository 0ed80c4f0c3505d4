"""End-to-end parity of the HIP encoder + head against the CPU fp32 oracle.

Bar: per image max|Δlogit| / max|logit_ref| <= 1e-3 and identical
per-segment argmax labels, where the margin between the oracle's top-1 and top-2 exceeds the
measured error (near-ties are reported, not asserted). Embeddings: cosine(f_gpu, f_ref).
"""
import numpy as np
import pytest
import torch

from interior_amd import config as C
from interior_amd.engine import VisionEngine
from interior_amd.lora import synthetic_adapters
from interior_amd.weights import synthetic_state_dict
from oracle import clip_ref

pytestmark = pytest.mark.gpu

# 1e-3 relative is the BASELINE bar; fp16 operands (the default, and the reference's own CUDA
# dtype) meet it in every config. bf16 (8-bit mantissa) does NOT: measured ~1.4e-3 at realistic
# logit scale and ~4.4e-3 against random text rows, so its checks use the looser bounds below
# (DESIGN.md §3).
LOGIT_TOL = {("bf16", "peaked"): 2e-3, ("fp16", "peaked"): 1e-3,
             ("bf16", "random"): 6e-3, ("fp16", "random"): 1e-3}
PROB_TOL = {"bf16": 2e-2, "fp16": 5e-3}


def _pixels(B, R, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, 3, R, R, generator=g).clamp_(-1.8, 2.2)


def _text(E, C_, seed=5, anchor=None, a=0.3):
    """Unit text rows. ``anchor`` (a unit image-feature direction from held-out images) gives
    realistically peaked logits: cos(f, T_c) ~ a, i.e. 100*cos ~ 30 like real CLIP
    image-prompt pairs (SURVEY.md §7 'Hard parts'); without it rows are random (logits ~ +-5,
    the hardest case for a relative bar)."""
    g = torch.Generator().manual_seed(seed)
    T = torch.randn(C_, E, generator=g)
    T = T / T.norm(dim=-1, keepdim=True)
    if anchor is not None:
        T = a * anchor[None, :] + (1 - a * a) ** 0.5 * T
        T = T / T.norm(dim=-1, keepdim=True)
    return T


def _anchor(ref_sd, name, R):
    f = clip_ref.encode_image(ref_sd, clip_ref.GEOMETRIES[name], _pixels(4, R, seed=999))
    m = (f / f.norm(dim=-1, keepdim=True)).mean(0)
    return m / m.norm()


def _merged(sd, adapters):
    out = dict(sd)
    for a in adapters:
        out[a.target] = clip_ref.merge_lora(sd[a.target], torch.from_numpy(a.A), torch.from_numpy(a.B),
                                            a.scaling)
    return out


_ENGINES = {}


def _fc_tiles(eng):
    """Tile variants of the c_fc launches logged since the last call (tuning trace_gemm=1)."""
    return sorted({v for role, v, _, _ in eng.gemm_log() if role == 2})


def _engine(cfg, dtype, lora_rank=0, max_batch=256):
    key = (cfg.name, dtype, lora_rank, max_batch)
    if key not in _ENGINES:
        sd = synthetic_state_dict(cfg, 0)
        eng = VisionEngine(cfg, 0, dtype, max_batch)
        eng.load_state_dict(sd)
        ref_sd = sd
        if lora_rank:
            ad = synthetic_adapters(cfg, rank=lora_rank)
            eng.load_lora(ad)
            ref_sd = _merged(sd, ad)
        _ENGINES[key] = (eng, ref_sd)
    return _ENGINES[key]


def _check_logits(lg, lr, seg, tol):
    rel = (np.abs(lg - lr).max(axis=1) / np.abs(lr).max(axis=1))
    assert rel.max() <= tol, f"max rel logit err {rel.max():.2e} > {tol}"
    bad = []
    for s in range(len(seg) - 1):
        a, b = seg[s], seg[s + 1]
        top_r = lr[:, a:b].argmax(1)
        top_g = lg[:, a:b].argmax(1)
        srt = np.sort(lr[:, a:b], axis=1)
        margin = srt[:, -1] - srt[:, -2] if b - a > 1 else np.full(len(lr), np.inf)
        err = np.abs(lg - lr)[:, a:b].max(1)
        decided = margin > 2 * err
        bad += [(i, s) for i in np.nonzero(decided & (top_r != top_g))[0]]
    assert not bad, f"argmax differs on decided rows: {bad[:5]}"
    return rel.max()


@pytest.mark.parametrize("text", ["peaked", "random"])
@pytest.mark.parametrize("name,dtype,B,lora", [
    ("ViT-B/32", "bf16", 8, 0),
    ("ViT-B/32", "bf16", 8, 8),
    ("ViT-B/32", "fp16", 8, 8),
    ("ViT-B/16", "bf16", 4, 0),
    ("ViT-B/16", "fp16", 4, 4),
    ("ViT-L/14@336px", "fp16", 2, 16),
])
def test_classify_matches_oracle(gpu, name, dtype, B, lora, text):
    cfg = C.get_config(name)
    eng, ref_sd = _engine(cfg, dtype, lora, max_batch=16)
    px = _pixels(B, cfg.image_size, seed=11)
    T = _text(cfg.embed_dim, 437, anchor=_anchor(ref_sd, name, cfg.image_size) if text == "peaked" else None)
    seg = [0, 40, 60, 359, 395, 425, 437]
    eng.set_text_features(T.numpy(), seg)
    out = eng.classify(px.to(gpu))
    torch.cuda.synchronize()
    f_ref = clip_ref.encode_image(ref_sd, clip_ref.GEOMETRIES[name], px)
    fh, lr, pr, ti, tp = clip_ref.head(f_ref, T, seg)
    cos = torch.nn.functional.cosine_similarity(out.emb.cpu(), fh, dim=-1)
    assert cos.min() > 0.9995, cos
    rel = _check_logits(out.logits.cpu().numpy(), lr.numpy(), seg, LOGIT_TOL[(dtype, text)])
    # probabilities within each segment
    assert np.abs(out.probs.cpu().numpy() - pr.numpy()).max() < PROB_TOL[dtype]
    print(f"{name} {dtype} lora={lora} text={text}: max|logit| {np.abs(lr.numpy()).max():.1f} "
          f"max rel logit err {rel:.2e}, min cos {cos.min():.7f}")


def test_encode_image_unnormalised(gpu):
    cfg = C.VIT_B32
    eng, ref_sd = _engine(cfg, "bf16", 0, max_batch=16)
    px = _pixels(3, 224, seed=2)
    f = eng.encode_image(px.to(gpu)).cpu()
    ref = clip_ref.encode_image(ref_sd, clip_ref.GEOMETRIES["ViT-B/32"], px)
    assert (f.norm(dim=-1) / ref.norm(dim=-1) - 1).abs().max() < 5e-3
    assert torch.nn.functional.cosine_similarity(f, ref).min() > 0.9995


def test_two_lane_split_is_bit_identical(gpu):
    """The two-stream split (default from 12,800 tokens per batch; tuning split_min) computes every image with the same
    kernels and k-order, so its outputs equal the single-stream outputs bit for bit."""
    cfg = C.VIT_B32
    sd = synthetic_state_dict(cfg, 0)
    T = _text(cfg.embed_dim, 437)
    seg = [0, 40, 60, 359, 395, 425, 437]
    px = _pixels(96, 224, seed=21).to(gpu)
    outs = []
    for split in ("0", "64"):
        eng = VisionEngine(cfg, 0, "fp16", max_batch=128, tuning={"split_min": split})
        eng.load_state_dict(sd)
        eng.set_text_features(T.numpy(), seg)
        o = eng.classify(px)
        torch.cuda.synchronize()
        outs.append((o.logits.clone(), o.top_idx.clone(), eng.encode_image(px).clone()))
        eng.close()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][2], outs[1][2])


def test_head_column_tile_is_bit_identical(gpu):
    """The head products (ln_post @ proj, 100 f_hat T^T) on 32-column workgroups (tuning
    head_cols=32) do every output element's arithmetic in the same order as on 64-column ones:
    features, logits, probabilities and top-k equal bit for bit (B = 67: a ragged 16-image group)."""
    cfg = C.VIT_B32
    sd = synthetic_state_dict(cfg, 0)
    T = _text(cfg.embed_dim, 437)
    seg = [0, 40, 60, 359, 395, 425, 437]
    px = _pixels(67, 224, seed=29).to(gpu)
    outs = []
    for cols in ("64", "32"):
        eng = VisionEngine(cfg, 0, "fp16", max_batch=67, tuning={"head_cols": cols})
        eng.load_state_dict(sd)
        eng.set_text_features(T.numpy(), seg)
        o = eng.classify(px)
        torch.cuda.synchronize()
        outs.append((o.logits.clone(), o.probs.clone(), o.top_idx.clone(), o.emb.clone(),
                     eng.encode_image(px).clone()))
        eng.close()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp16", "bf16"])
def test_cls_prune_and_deferred_adds_are_bit_identical(gpu, dtype):
    """The deferred residual store (tuning defer_x) executes the same per-row fp32 operations in
    the same order, so the features equal the full computation's bit for bit (B/32 and the
    N = 197 B/16 geometry), with the last block on class-token rows only (cls_prune) and
    without, with the LayerNorm fold (lnfold) and without. The unfolded class-token tail
    splits K of its three GEMMs (fp32 partials summed in slice order, no 16-bit branch output),
    so pruned and full last blocks agree to rounding; the folded tail stays bit-identical. The
    folded and unfolded paths agree to rounding (different but equivalent arithmetic). The
    identities hold for the fp32 residual stream (x24=0); the default 24-bit stream
    (pruned + deferred path) is compared with it to rounding."""
    for cfg, B in ((C.VIT_B32, 67), (C.VIT_B16, 9)):
        sd = synthetic_state_dict(cfg, 0)
        ad = synthetic_adapters(cfg, rank=8)
        px = _pixels(B, cfg.image_size, seed=23).to(gpu)
        groups = {}
        for fold, prune, defer in (("1", "0", "0"), ("1", "1", "0"), ("0", "0", "0"), ("0", "1", "1"),
                                   ("0", "1", "0"), ("0", "0", "1")):
            eng = VisionEngine(cfg, 0, dtype, max_batch=B,
                               tuning={"x24": 0, "lnfold": fold, "cls_prune": prune, "defer_x": defer})
            eng.load_state_dict(sd)
            eng.load_lora(ad)
            # the fold applies to the fp16 path only (bf16 ignores lnfold)
            key = "fold" if fold == "1" and dtype == "fp16" else "prune" + prune
            groups.setdefault(key, []).append(eng.encode_image(px).clone())
            torch.cuda.synchronize()
            eng.close()
        for key, outs in groups.items():
            for o in outs[1:]:
                assert torch.equal(outs[0], o), (cfg.name, dtype, key)

        def rel(a, b):
            return ((a - b).norm(dim=-1) / b.norm(dim=-1)).max().item()

        split = rel(groups["prune1"][0], groups["prune0"][0])
        assert split < (5e-4 if dtype == "fp16" else 5e-3), (cfg.name, dtype, split)
        print(f"[{cfg.name} {dtype}] split-K class-token tail vs full last block: rel {split:.2e}")
        if "fold" in groups:
            f1, f0 = groups["fold"][0], groups["prune0"][0]
            assert rel(f1, f0) < 3e-3, (cfg.name, dtype, rel(f1, f0))
        # the 24-bit residual stream (default): x rounded to a 16-bit significand at every store
        eng = VisionEngine(cfg, 0, dtype, max_batch=B)  # shipped defaults: x24, cls_prune, defer_x
        eng.load_state_dict(sd)
        eng.load_lora(ad)
        f24 = eng.encode_image(px).clone()
        eng.close()
        d24 = rel(f24, groups["prune1"][0])
        print(f"[{cfg.name} {dtype}] 24-bit vs fp32 residual stream: rel {d24:.2e}")
        assert 0 < d24 < (1.5e-3 if dtype == "fp16" else 1e-2), (cfg.name, dtype, d24)
        if "fold" in groups:  # the fold on the 24-bit stream (EPI_RES_STATS x24 planes)
            eng = VisionEngine(cfg, 0, dtype, max_batch=B, tuning={"lnfold": 1})
            eng.load_state_dict(sd)
            eng.load_lora(ad)
            g24 = eng.encode_image(px).clone()
            eng.close()
            e24 = rel(g24, groups["fold"][0])
            print(f"[{cfg.name} {dtype}] folded: 24-bit vs fp32 residual stream: rel {e24:.2e}")
            assert 0 < e24 < 1.5e-3, (cfg.name, dtype, e24)


@pytest.mark.parametrize("dtype,pdt", [("fp16", torch.float16), ("bf16", torch.bfloat16)])
def test_pixel_dtype_16bit_input_is_bit_identical(gpu, dtype, pdt):
    """The patch GEMM reads 16-bit pixels of the MFMA operand type (fp32 pixels are cast once);
    16-bit pixels of that type (what bench.py feeds, clip's image.type(model.dtype)) give
    bit-identical features."""
    cfg = C.VIT_B32
    eng, _ = _engine(cfg, dtype, lora_rank=8, max_batch=256)
    px = _pixels(33, 224, seed=29).to(gpu)
    a = eng.encode_image(px).clone()
    b = eng.encode_image(px.to(pdt)).clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_batches_in_flight_on_two_streams(gpu):
    """bench.py keeps two batches in flight on two HIP streams; the handle gives the second
    in-flight call its own workspace. Outputs equal the single-stream outputs bit for bit."""
    cfg = C.VIT_B32
    sd = synthetic_state_dict(cfg, 0)
    T = _text(cfg.embed_dim, 437)
    seg = [0, 40, 60, 359, 395, 425, 437]
    eng = VisionEngine(cfg, 0, "fp16", max_batch=128)
    eng.load_state_dict(sd)
    eng.set_text_features(T.numpy(), seg)
    pxs = [_pixels(96, 224, seed=31 + i).to(gpu) for i in range(4)]
    ref = [eng.classify(p).logits.clone() for p in pxs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)]
    outs = [None] * 4
    for i, p in enumerate(pxs):
        with torch.cuda.stream(streams[i % 2]):
            outs[i] = eng.classify(p)
    torch.cuda.synchronize()
    for r, o in zip(ref, outs):
        assert torch.equal(r, o.logits)
    eng.close()


def test_concurrent_host_threads(gpu):
    """The reference calls encode_image from ThreadPoolExecutor(4) (main.py:345-346); the
    handle must give every thread its own workspace and correct results."""
    from concurrent.futures import ThreadPoolExecutor
    cfg = C.VIT_B32
    eng, ref_sd = _engine(cfg, "fp16", 0, max_batch=16)
    pxs = [_pixels(3, 224, seed=100 + i).to(gpu) for i in range(8)]
    serial = [eng.encode_image(p).clone() for p in pxs]
    torch.cuda.synchronize()

    def work(i):
        s = torch.cuda.Stream(gpu)
        with torch.cuda.stream(s):
            out = eng.encode_image(pxs[i])
        s.synchronize()
        return out

    with ThreadPoolExecutor(max_workers=4) as ex:
        par = list(ex.map(work, range(8)))
    for a, b in zip(serial, par):
        assert torch.equal(a, b)


def test_errors_are_reported_not_crashes(gpu):
    from interior_amd import _lib
    cfg = C.VIT_B32
    eng, _ = _engine(cfg, "fp16", 0, max_batch=16)
    with pytest.raises(_lib.ClipVitError):
        eng.encode_image(torch.zeros(17, 3, 224, 224, device=gpu)[:0])  # B = 0
    eng2 = VisionEngine(cfg, 0, "fp16", 4)
    with pytest.raises(_lib.ClipVitError):
        eng2.encode_image(torch.zeros(1, 3, 224, 224, device=gpu))     # weights not loaded
    eng2.close()


@pytest.mark.parametrize("dtype", ["fp16", "bf16"])
def test_full_batch_256_properties(gpu, dtype):
    """bs=256 (the metric's batch; c_fc as ONE balanced launch of variant 75, the fp16 default):
    every image equals its own bs=1 result bit-for-bit (per-image independence; rows never mix),
    and a sample of rows matches the oracle."""
    cfg = C.VIT_B32
    eng, ref_sd = _engine(cfg, dtype, 8, max_batch=256)
    px = _pixels(256, 224, seed=3).to(gpu)
    T = _text(cfg.embed_dim, 437, anchor=_anchor(ref_sd, "ViT-B/32", 224))
    seg = [0, 40, 60, 359, 395, 425, 437]
    eng.set_text_features(T.numpy(), seg)
    full = eng.classify(px).logits.clone()
    for i in (0, 1, 77, 230, 255):
        one = eng.classify(px[i:i + 1]).logits
        assert torch.equal(one[0], full[i]), i
    idx = [0, 100, 215, 255]  # first, middle and last images (v75 tiles of all three rounds)
    f_ref = clip_ref.encode_image(ref_sd, clip_ref.GEOMETRIES["ViT-B/32"], px[idx].cpu())
    _, lr, _, _, _ = clip_ref.head(f_ref, T, seg)
    _check_logits(full[idx].cpu().numpy(), lr.numpy(), seg, LOGIT_TOL[(dtype, "peaked")])


def test_b32_bs128_round_split_matches_oracle(gpu):
    """B/32 fp16 bs 128: c_fc's 300 tiles = 1 round + 44, where the whole-round row split is the
    default (v62 on rows [0, 5376), v81 on the rest). The launch log pins that
    path; rows of both launches against the oracle at the 1e-3 bar, and the split against the
    single-launch tile (round_split=0) bit for bit."""
    cfg = C.VIT_B32
    sd = synthetic_state_dict(cfg, 0)
    ad = synthetic_adapters(cfg, rank=8)
    ref_sd = _merged(sd, ad)
    px = _pixels(128, 224, seed=45)
    T = _text(cfg.embed_dim, 437, anchor=_anchor(ref_sd, cfg.name, 224))
    seg = [0, 40, 60, 359, 395, 425, 437]
    outs, tiles = {}, {}
    for split in (1, 0):
        eng = VisionEngine(cfg, 0, "fp16", max_batch=128, tuning={"trace_gemm": 1, "round_split": split})
        try:
            eng.load_state_dict(sd)
            eng.load_lora(ad)
            eng.set_text_features(T.numpy(), seg)
            eng.gemm_log()
            outs[split] = eng.classify(px.to(gpu)).logits.clone()
            torch.cuda.synchronize()
            tiles[split] = _fc_tiles(eng)
        finally:
            eng.close()
    assert tiles[1] == [62, 81], tiles
    assert tiles[0] == [22], tiles
    assert torch.equal(outs[0], outs[1])
    idx = [0, 64, 110, 127]  # 110, 127: rows >= 5376 (image 107.5 on), the v81 launch
    f_ref = clip_ref.encode_image(ref_sd, clip_ref.GEOMETRIES[cfg.name], px[idx])
    _, lr, _, _, _ = clip_ref.head(f_ref, T, seg)
    rel = _check_logits(outs[1][idx].cpu().numpy(), lr.numpy(), seg, LOGIT_TOL[("fp16", "peaked")])
    print(f"B/32 bs 128 (v62 + v81 c_fc): max rel logit err {rel:.2e} on rows {idx}")


def test_config4_l14_336_bs128_as_benched(gpu):
    """BASELINE config 4 exactly as bench.py runs it: ViT-L/14@336 + merged LoRA r=16, fp16, 128
    images in one classify, which takes the two-lane half-batch split (64 images per lane stream)
    and the 256x256 v80 tiles of every role. A sample of rows from both lanes against the oracle
    at the 1e-3 bar (peaked text), and the split against one stream bit for bit (VERDICT r02
    item 4; main.py:440-448 batches the same way)."""
    cfg = C.get_config("ViT-L/14@336px")
    sd = synthetic_state_dict(cfg, 0)
    ad = synthetic_adapters(cfg, rank=16)
    ref_sd = _merged(sd, ad)
    px = _pixels(128, cfg.image_size, seed=41)
    T = _text(cfg.embed_dim, 437, anchor=_anchor(ref_sd, cfg.name, cfg.image_size))
    seg = [0, 40, 60, 359, 395, 425, 437]
    outs = {}
    for split in ("default", "0"):
        eng = VisionEngine(cfg, 0, "fp16", max_batch=128, tuning=None if split == "default" else {"split_min": split})
        eng.load_state_dict(sd)
        eng.load_lora(ad)
        eng.set_text_features(T.numpy(), seg)
        o = eng.classify(px.to(gpu))
        torch.cuda.synchronize()
        outs[split] = (o.logits.clone(), o.top_idx.clone(), o.emb.clone())
        eng.close()
    for a, b in zip(outs["default"], outs["0"]):
        assert torch.equal(a, b)
    idx = [0, 63, 64, 127]  # first and last image of each lane
    f_ref = clip_ref.encode_image(ref_sd, clip_ref.GEOMETRIES[cfg.name], px[idx])
    _, lr, _, _, _ = clip_ref.head(f_ref, T, seg)
    rel = _check_logits(outs["default"][0][idx].cpu().numpy(), lr.numpy(), seg, LOGIT_TOL[("fp16", "peaked")])
    print(f"L/14@336 bs 128 (split + v80 tiles): max rel logit err {rel:.2e} on rows {idx}")


@pytest.mark.parametrize("x24", [1, 0])
def test_lnfold_bs256_takes_the_single_launch(gpu, x24):
    """the LayerNorm-fold path (tuning lnfold=1) at the headline batch, B/32 bs 256.
    The balanced v75 launch and the ping-pong round-split tiles have only the 16-bit STORE / GELU
    epilogues, so the folded c_fc (EPI_LNF_GELU) must take the single-launch v22 tile instead of
    failing (the launch log pins it). Rows from the start, middle and end of the batch against
    the oracle at the 1e-3 bar (peaked text), on the 24-bit residual stream and on fp32 x."""
    cfg = C.VIT_B32
    sd = synthetic_state_dict(cfg, 0)
    ad = synthetic_adapters(cfg, rank=8)
    ref_sd = _merged(sd, ad)
    px = _pixels(256, 224, seed=43)
    T = _text(cfg.embed_dim, 437, anchor=_anchor(ref_sd, cfg.name, 224))
    seg = [0, 40, 60, 359, 395, 425, 437]
    eng = VisionEngine(cfg, 0, "fp16", max_batch=256, tuning={"lnfold": 1, "x24": x24, "trace_gemm": 1})
    try:
        eng.load_state_dict(sd)
        eng.load_lora(ad)
        eng.set_text_features(T.numpy(), seg)
        eng.gemm_log()
        o = eng.classify(px.to(gpu))
        torch.cuda.synchronize()
        assert _fc_tiles(eng) == [22]
        idx = [0, 127, 214, 255]
        f_ref = clip_ref.encode_image(ref_sd, clip_ref.GEOMETRIES[cfg.name], px[idx])
        _, lr, _, _, _ = clip_ref.head(f_ref, T, seg)
        rel = _check_logits(o.logits[idx].cpu().numpy(), lr.numpy(), seg, LOGIT_TOL[("fp16", "peaked")])
        print(f"B/32 bs 256 lnfold x24={x24}: max rel logit err {rel:.2e}")
    finally:
        eng.close()


# c_fc tile variants each row must reach (the launch log, tuning trace_gemm=1): 75 = the balanced
# one-launch tile, 62 + 81 / 72 + 81 / 74 + 81 = round split main + tail, 22 = one launch on the
# 160x128 tile, 74 / 8 = large-M tiles, 3 = the MX-fp8 persistent tile
@pytest.mark.parametrize("name,dtype,B,tun,fc", [
    ("ViT-B/32", "fp16", 256, {}, [75]),        # c_fc: one balanced launch (default); c_proj v82
    ("ViT-B/32", "fp16", 256, {"split_variants": "72,81", "fc_balanced": 0}, [72, 81]),  # 32-deep-k-step main
    ("ViT-B/32", "fp16", 256, {"fc_balanced": 0}, [62, 81]),  # the round split: ping-pong main + tail
    ("ViT-B/32", "fp16", 128, {}, [62, 81]),    # bs 128: 1 round + 44 tiles, the round split by default
    ("ViT-B/32", "bf16", 67, {}, [22]),         # one launch per role
    ("ViT-B/32", "fp16", 1, {}, [22]),          # M = 50: the last 16-row block is padding
    ("ViT-B/32", "fp16", 256, {"lnfold": 1}, [22]),  # EPI_LNF_GELU c_fc, EPI_RES_STATS c_proj
    ("ViT-B/32", "fp16", 256, {"split_variants": "74,81", "fc_balanced": 0}, [74, 81]),  # non-temporal main
    ("ViT-B/16", "fp16", 64, {}, [75]),         # N = 197: 600 tiles, balanced launch
    ("ViT-B/16", "fp16", 64, {"fc_balanced": 0}, [62, 81]),  # N = 197, round split
    ("ViT-L/14@336px", "fp16", 32, {}, [74]),   # large M: persistent v74 writes u, v72 reads it
    ("ViT-L/14@336px", "fp16", 32, {"large_variants": "3462,8,3462,8"}, [8]),  # v8 direct stores, v62 / v8 read
    ("ViT-B/32", "mxfp8", 64, {}, [3, 22]),     # MX-fp8: fp8 u of the MX blocks, 16-bit u of the rest
    ("ViT-B/32", "mxfp8", 64, {"mx8_skip": ""}, [3]),  # every block MX; the last c_proj keeps u row-major
])
def test_blocked_u_is_bit_identical(gpu, name, dtype, B, tun, fc):
    """The c_fc -> c_proj intermediate in the 16-row blocked layout (default; tuning u_blocked=0:
    row-major) moves bytes only: every kernel computes the same values in the same order, so the
    features equal the row-major run's bit for bit on every GEMM path that writes or reads u.
    The launch log pins the c_fc tiles each row reaches."""
    cfg = C.get_config(name)
    sd = synthetic_state_dict(cfg, 0)
    ad = synthetic_adapters(cfg, rank=8)
    px = _pixels(B, cfg.image_size, seed=47).to(gpu)
    outs = []
    for blk in (1, 0):
        eng = VisionEngine(cfg, 0, dtype, max_batch=B, tuning=dict(tun, u_blocked=blk, trace_gemm=1))
        try:
            eng.load_state_dict(sd)
            eng.load_lora(ad)
            eng.gemm_log()
            outs.append(eng.encode_image(px).clone())
            torch.cuda.synchronize()
            log = eng.gemm_log()
            assert sorted({v for r, v, _, _ in log if r == 2}) == fc, (tun, log)
            if blk:  # the blocked u is written by c_fc and read by c_proj on every full-M launch
                assert any(r == 2 and f & 8 for r, _, _, f in log) and any(r == 3 and f & 4 for r, _, _, f in log)
        finally:
            eng.close()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]), (name, dtype, B, tun)


@pytest.mark.parametrize("name,dtype,B,tun,fc", [
    ("ViT-B/32", "fp16", 256, {}, [75]),                      # QKV v72, c_fc v75, out / c_proj v82: all read the copy (2)
    ("ViT-B/32", "fp16", 256, {"split_variants": "72,81", "fc_balanced": 0}, [72, 81]),  # c_fc main 72 + tail 81
    ("ViT-B/32", "fp16", 256, {"fc_balanced": 0}, [62, 81]),  # the round split (v62 reads the copy, the tail follows it)
    ("ViT-B/32", "fp16", 128, {}, [62, 81]),                  # bs 128: the round split by default
    ("ViT-B/32", "bf16", 67, {"qkv_variant": "72"}, [22]),    # one launch per role, ragged M
    ("ViT-B/16", "fp16", 64, {}, [75]),                       # N = 197, balanced c_fc launch
    ("ViT-B/16", "fp16", 256, {}, [74]),                      # large M: every role on 3472, c_fc 3474 (default)
    ("ViT-L/14@336px", "fp16", 32, {}, [74]),                 # large M: c_fc on the shipped 3474
    ("ViT-L/14@336px", "fp16", 64, {}, [74]),                 # every role large-M: 3472 / 3474, blocked A
    ("ViT-L/14@336px", "fp16", 32, {"large_variants": "3408,8,3462,8"}, [8]),  # large-M pipelined / ping-pong tiles
])
def test_blocked_w_is_bit_identical(gpu, name, dtype, B, tun, fc):
    """The Linear weights read from their 16-row blocked copy (tuning w_blocked: 2 = every tile
    that can, the default; 1 = the variant-72 / 74 launches only; 0 = none) move bytes only:
    every tile computes the same products in the same order, so the features equal the
    row-major run's (w_blocked=0) bit for bit — after a LoRA merge, which re-packs both copies.
    The launch log pins the c_fc tiles of each row and that w_blocked=0 reads no copy."""
    cfg = C.get_config(name)
    sd = synthetic_state_dict(cfg, 0)
    ad = synthetic_adapters(cfg, rank=8)
    px = _pixels(B, cfg.image_size, seed=53).to(gpu)
    outs = []
    for blk in (2, 1, 0):
        # attn_fuse=0: the fused attention sub-block reads only the blocked W_out copy, so the
        # layouts are compared on the three-kernel path (test_attention_block_fusion covers it)
        eng = VisionEngine(cfg, 0, dtype, max_batch=B, tuning=dict(tun, w_blocked=blk, trace_gemm=1, attn_fuse=0))
        try:
            eng.load_state_dict(sd)
            eng.load_lora(ad)
            eng.gemm_log()
            outs.append(eng.encode_image(px).clone())
            torch.cuda.synchronize()
            log = eng.gemm_log()
            assert sorted({v for r, v, _, _ in log if r == 2}) == fc, (tun, blk, log)
            copies = sum(1 for _, _, _, f in log if f & 1)
            want = blk == 2 or (blk == 1 and any(v in (72, 74) for _, v, _, _ in log))
            assert (copies > 0) == want, (blk, log)
        finally:
            eng.close()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[2]), (name, dtype, B, tun)


@pytest.mark.parametrize("hmode", [1, 2, 3])
@pytest.mark.parametrize("name,dtype,B,tun", [
    ("ViT-B/32", "fp16", 256, {}),                 # c_fc v75
    ("ViT-B/32", "fp16", 128, {}),                 # c_fc round split v62 + v81
    ("ViT-B/32", "bf16", 67, {}),                  # ragged M: the last 16-row group is part padding
    ("ViT-B/32", "fp16", 1, {}),                   # M = 50
    ("ViT-B/16", "fp16", 256, {}),                 # two lanes, large-M tile 3474
    ("ViT-L/14@336px", "fp16", 32, {}),            # D = 1024
])
def test_blocked_h_is_bit_identical(gpu, name, dtype, B, tun, hmode):
    """ln_2's output h in the 16-row blocked layout (tuning h_blocked: 1 = direct stores, 2 / 3 = an
    LDS transpose of 16 / 8 rows in the LN kernel; c_fc stages 1 KB runs) moves bytes only: the
    features equal the row-major run's bit for bit, and the launch log shows c_fc reading a blocked
    A (and QKV from block 1, qkv_blk) exactly when h_blocked is on."""
    cfg = C.get_config(name)
    sd = synthetic_state_dict(cfg, 0)
    ad = synthetic_adapters(cfg, rank=8)
    px = _pixels(B, cfg.image_size, seed=59).to(gpu)
    outs = []
    for hb in (hmode, 0):
        # attn_fuse=0: the fused attention sub-block writes blocked h itself (h_blocked != 0 only)
        eng = VisionEngine(cfg, 0, dtype, max_batch=B, tuning=dict(tun, h_blocked=hb, trace_gemm=1, attn_fuse=0))
        try:
            eng.load_state_dict(sd)
            eng.load_lora(ad)
            eng.gemm_log()
            outs.append(eng.encode_image(px).clone())
            torch.cuda.synchronize()
            log = eng.gemm_log()
            assert {bool(f & 4) for r, _, _, f in log if r == 2} == {bool(hb)}, (hb, log)  # c_fc
            qkv = [bool(f & 4) for r, _, _, f in log if r == 0]  # QKV: blocked from block 1 (qkv_blk)
            assert any(qkv) == bool(hb) and not all(qkv), (hb, log)
        finally:
            eng.close()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]), (name, dtype, B, tun)


@pytest.mark.parametrize("name,dtype,B,pix16", [
    ("ViT-B/32", "fp16", 256, False),   # fp32 pixels (the bench): cast pass -> blocked im2col
    ("ViT-B/32", "bf16", 67, False),    # ragged M = 67 * 49: the last 16-row block is part padding
    ("ViT-B/32", "fp16", 1, False),     # M = 49
    ("ViT-B/16", "fp16", 130, False),   # two lanes, P = 16
    ("ViT-L/14@336px", "fp16", 8, False),  # P = 14: patch rows padded to 16 pixels, Kp = 704
    ("ViT-L/14@336px", "fp16", 8, True),   # 16-bit pixels, P = 14: the padded cast ran anyway
])
def test_patch_im2col_is_bit_identical(gpu, name, dtype, B, pix16):
    """The explicit patch GEMM (tuning patch_im2col: blocked im2col written by the cast pass, then
    the pipelined 160x128 tile on blocked A and W) uses the implicit GEMM's k order and k-tile
    sequence, so the features equal the implicit GEMM's bit for bit."""
    cfg = C.get_config(name)
    sd = synthetic_state_dict(cfg, 0)
    px = _pixels(B, cfg.image_size, seed=61).to(gpu)
    if pix16:
        px = px.to(torch.float16 if dtype == "fp16" else torch.bfloat16)
    outs = []
    for im2col in (1, 0):
        eng = VisionEngine(cfg, 0, dtype, max_batch=B, tuning=dict(patch_im2col=im2col))
        try:
            eng.load_state_dict(sd)
            outs.append(eng.encode_image(px).clone())
            torch.cuda.synchronize()
        finally:
            eng.close()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]), (name, dtype, B)


@pytest.mark.parametrize("dtype,persist", [("fp16", 2), ("bf16", 1), ("mxfp8", 2)])
def test_attention_persistent_engine_bit_identical(gpu, dtype, persist):
    """ViT-B/32 (N = 50) with the persistent one-key-block attention (tuning attn_persist; for
    MX-fp8 its quantizing epilogue) gives the same features as the one-workgroup-per-unit kernel,
    bit for bit."""
    cfg = C.get_config("ViT-B/32")
    sd = synthetic_state_dict(cfg, 0)
    px = _pixels(64, cfg.image_size, seed=67).to(gpu)
    outs = []
    for p in (persist, 0):
        eng = VisionEngine(cfg, 0, dtype, max_batch=64, tuning=dict(attn_persist=p, attn_fuse=0))
        try:
            eng.load_state_dict(sd)
            outs.append(eng.encode_image(px).clone())
            torch.cuda.synchronize()
        finally:
            eng.close()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]), (dtype, persist)


@pytest.mark.parametrize("name,dtype,B", [("ViT-B/32", "fp16", 256), ("ViT-B/32", "bf16", 67), ("ViT-B/16", "fp16", 33)])
def test_ln1_rows_is_bit_identical(gpu, name, dtype, B):
    """The add + LayerNorm after c_proj with two rows per wave (tuning ln1_rows=2; ragged row
    counts leave the last wave one row) does each row's arithmetic as with one: same features."""
    cfg = C.get_config(name)
    sd = synthetic_state_dict(cfg, 0)
    px = _pixels(B, cfg.image_size, seed=71).to(gpu)
    outs = []
    for r in (2, 1):
        eng = VisionEngine(cfg, 0, dtype, max_batch=B, tuning=dict(ln1_rows=r, attn_fuse=0))
        try:
            eng.load_state_dict(sd)
            outs.append(eng.encode_image(px).clone())
            torch.cuda.synchronize()
        finally:
            eng.close()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]), (name, dtype, B)


@pytest.mark.parametrize("name,dtype,B,tun", [
    ("ViT-B/32", "fp16", 256, {}),                      # QKV v98 (pipelined 240x256) on blocked A
    ("ViT-B/32", "fp16", 256, {"qkv_variant": 72}),     # QKV on the 32-deep-k-step tile
    ("ViT-B/32", "bf16", 67, {"qkv_variant": 72}),      # ragged M
    ("ViT-B/16", "fp16", 256, {}),                      # two lanes, large-M tile
    ("ViT-L/14@336px", "fp16", 32, {}),                 # D = 1024
])
def test_blocked_qkv_h_is_bit_identical(gpu, name, dtype, B, tun):
    """ln_1 (the add + LayerNorm after c_proj) writing QKV's A in the 16-row blocked layout
    (tuning qkv_blk; block 0's h stays row-major from embed_ln) moves bytes only: the features
    equal the row-major run's bit for bit, and the launch log shows blocked-A QKV launches only
    with the option on."""
    cfg = C.get_config(name)
    sd = synthetic_state_dict(cfg, 0)
    px = _pixels(B, cfg.image_size, seed=73).to(gpu)
    outs = []
    for qb in (1, 0):
        eng = VisionEngine(cfg, 0, dtype, max_batch=B, tuning=dict(tun, qkv_blk=qb, trace_gemm=1))
        try:
            eng.load_state_dict(sd)
            eng.gemm_log()
            outs.append(eng.encode_image(px).clone())
            torch.cuda.synchronize()
            flags = [bool(f & 4) for r, _, _, f in eng.gemm_log() if r == 0]
            assert any(flags) == bool(qb) and not all(flags), (qb, flags)
        finally:
            eng.close()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1]), (name, dtype, B, tun)


@pytest.mark.parametrize("dtype,B", [("fp16", 256), ("fp16", 1), ("bf16", 67)])
def test_attention_block_fusion(gpu, dtype, B):
    """ViT-B/32 blocks 0 .. L-2 as one kernel per image (attention + out_proj + x += y + ln_2,
    attn_block.hip; the default) against the three-kernel path (tuning attn_fuse=0): the same
    products in another summation order, and x + y rounded once more to the 24-bit stream, so
    the features agree to a few fp16 ulps, not bit for bit; both against the CPU oracle at the
    1e-3 logit bar (fp16). Per image the fused kernel is independent of the batch: image 0 of a
    bs-B run equals the bs-1 run's bit for bit."""
    cfg = C.get_config("ViT-B/32")
    sd = synthetic_state_dict(cfg, 0)
    ad = synthetic_adapters(cfg, rank=8)
    px = _pixels(B, cfg.image_size, seed=79).to(gpu)
    feats = {}
    for fuse in (1, 0):
        eng = VisionEngine(cfg, 0, dtype, max_batch=B, tuning=dict(attn_fuse=fuse))
        try:
            eng.load_state_dict(sd)
            eng.load_lora(ad)
            feats[fuse] = eng.encode_image(px).clone()
            if fuse and B > 1:
                one = eng.encode_image(px[:1].contiguous()).clone()
                assert torch.equal(one[0], feats[fuse][0])
            torch.cuda.synchronize()
        finally:
            eng.close()
    f1, f0 = feats[1].float(), feats[0].float()
    assert torch.isfinite(f1).all()
    rel = ((f1 - f0).abs().amax(dim=1) / f0.abs().amax(dim=1)).max().item()
    assert rel <= (2e-3 if dtype == "fp16" else 2e-2), rel
    if dtype == "fp16":
        ref_sd = dict(sd)
        for a in ad:
            ref_sd[a.target] = clip_ref.merge_lora(sd[a.target], torch.from_numpy(a.A), torch.from_numpy(a.B), a.scaling)
        n = min(B, 4)
        ref = clip_ref.encode_image(ref_sd, clip_ref.GEOMETRIES[cfg.name], px[:n].cpu())
        err = [((f[:n].cpu() - ref).abs().amax(dim=1) / ref.abs().amax(dim=1)).max().item() for f in (f1, f0)]
        assert err[0] <= 1.25 * err[1] + 1e-4, err  # fused vs the oracle: no worse than the three kernels
        assert torch.nn.functional.cosine_similarity(f1[:n].cpu(), ref).min() > 0.9995

