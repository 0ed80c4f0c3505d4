"""MX-fp8 path (BASELINE.json config 5: fp8 weights, bf16 activations) on the GPU.

Pinned pieces:
  * quantizer: block scales equal the host restatement of the rule exactly, and every element
    equals the host round-to-nearest-even e4m3 of x * 2^-e (bit-exact);
  * GEMM: against fp64 A_deq @ W_deq^T (+ bias) of the SAME quantized operands — products of
    e4m3 values and power-of-two scales are exact, so only fp32 summation order differs
    (tolerance 1e-4 of max|C|: the scaled MFMA sums 128 products per instruction); integer-valued operands are checked for exact equality;
    the MX-fp8 / bf16 output epilogues equal the quantization / rounding of the fp32 one;
  * end to end: logits of the MX-fp8 engine within 2e-2 of the bf16 engine on the same weights
    (the config-5 bar, relative to max|logit|), and vs the fp32 oracle.
"""
import numpy as np
import pytest
import torch

from interior_amd import config as C
from interior_amd import engine as E
from interior_amd.engine import VisionEngine
from interior_amd.lora import synthetic_adapters
from interior_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


# ---------------------------------------------------------------- host restatement of MX-fp8
def _e4m3_table() -> np.ndarray:
    t = np.zeros(256, dtype=np.float64)
    for b in range(256):
        s, e, m = b >> 7, (b >> 3) & 15, b & 7
        v = (m / 8.0) * 2.0 ** -6 if e == 0 else (1 + m / 8.0) * 2.0 ** (e - 7)
        if e == 15 and m == 7:
            v = np.nan
        t[b] = -v if s else v
    return t


E4M3 = _e4m3_table()


def _block_exp(amax: np.ndarray) -> np.ndarray:
    """Smallest e with amax * 2^-e <= 448, clamped to [-127, 126]; amax == 0 -> -127."""
    with np.errstate(divide="ignore"):
        e = np.ceil(np.log2(amax.astype(np.float64) / 448.0))
    e = np.where(amax > 0, e, -127)
    return np.clip(e, -127, 126).astype(np.int64)


def _rne_e4m3(y: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even onto the e4m3 grid (|y| <= 448 by construction)."""
    a = np.abs(y.astype(np.float64))
    ex = np.floor(np.log2(np.where(a > 0, a, 1.0)))
    step = np.where(a < 2.0 ** -6, 2.0 ** -9, 2.0 ** (ex - 3))
    return np.sign(y) * np.round(a / step) * step  # np.round = half-to-even


def _dequant(q: torch.Tensor, s: torch.Tensor) -> np.ndarray:
    qv = E4M3[q.cpu().numpy().astype(np.int64)]
    sv = 2.0 ** (s.cpu().numpy().astype(np.float64) - 127)
    return qv * np.repeat(sv, 32, axis=1)


def _quant_host(x: np.ndarray):
    r, k = x.shape
    blocks = x.astype(np.float64).reshape(r, k // 32, 32)
    e = _block_exp(np.abs(blocks).max(-1))
    y = _rne_e4m3(blocks * 2.0 ** (-e[..., None]))
    return (y * 2.0 ** e[..., None]).reshape(r, k), (e + 127).astype(np.uint8)


# ---------------------------------------------------------------- quantizer
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_quant_mx8_matches_host_rule(gpu, dtype):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(97, 256, generator=g)
    x *= torch.logspace(-6, 4, 97)[:, None]           # every row a different magnitude
    x[5, :32] = 0.0                                    # an all-zero block
    x[6, 40] = 448.0 * 2 ** 3                          # exact power-of-two boundary
    x[7, 64:96] = torch.linspace(-1e-3, 1e-3, 32)      # values that land in the subnormal range
    x = x.to(dtype)
    q, s = E.quant_mx8_test(x.to(gpu))
    ref, ref_s = _quant_host(x.float().numpy())
    assert np.array_equal(s.cpu().numpy(), ref_s)
    got = _dequant(q, s)
    assert np.array_equal(got, ref), np.abs(got - ref).max()


# ---------------------------------------------------------------- GEMM
def _quantized_operands(gpu, M, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(M, K, generator=g)
    W = torch.randn(N, K, generator=g) * 0.05
    bias = torch.randn(N, generator=g)
    A8, sA = E.quant_mx8_test(A.to(gpu))
    W8, sW = E.quant_mx8_test(W.to(gpu))
    return A8, sA, W.to(gpu), bias.to(gpu), _dequant(A8, sA), _dequant(W8, sW)


@pytest.mark.parametrize("variant", [1, 2, 5, 201])
@pytest.mark.parametrize("M,N,K", [(12800, 768, 768), (1000, 2304, 768), (333, 3072, 768),
                                   (700, 768, 3072), (64, 256, 128), (130, 128, 256)])
def test_gemm_mx8_vs_dequantized_reference(gpu, variant, M, N, K):
    if variant % 100 == 1 and N % 256:
        pytest.skip("128x256 tile needs N % 256 == 0")
    A8, sA, W, bias, Ad, Wd = _quantized_operands(gpu, M, N, K, M + N + K)
    Cg = E.gemm_mx8_test(A8, sA, W, bias, epi=0, variant=variant).cpu().numpy()
    ref = Ad @ Wd.T + bias.cpu().numpy()[None, :]
    err = np.abs(Cg - ref).max() / np.abs(ref).max()
    assert err < 1e-4, err


@pytest.mark.parametrize("variant", [2, 3, 5])
@pytest.mark.parametrize("M,N,K", [(12800, 3072, 768), (12800, 768, 768), (1000, 2304, 768), (333, 3072, 768),
                                   (700, 768, 3072), (257, 512, 256)])
def test_gemm_mx8_ping_pong_bit_identical(gpu, variant, M, N, K):
    """The persistent 256x256 ping-pong MX tile (3), the 128x128 tile (2, the MX c_fc round
    split's tail launch) and the 160x128
    tile (5, two scale dwords per thread) accumulate every output in the same k order as the
    128x256 tile: their bf16 store and MX-fp8 (QuickGELU) output must be bit-identical to
    variant 1's, over repeated launches (race screen, as test_gpu_kernels.py's ping-pong
    screen)."""
    A8, sA, W, bias, Ad, Wd = _quantized_operands(gpu, M, N, K, M + N + K + 1)
    ref5 = E.gemm_mx8_test(A8, sA, W, bias, epi=5, variant=1)
    ref4 = E.gemm_mx8_test(A8, sA, W, bias, epi=4, variant=1)
    ref = torch.from_numpy(Ad @ Wd.T).float() + bias.cpu()[None, :]
    assert ((ref5.cpu().float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    for rep in range(3):
        got5 = E.gemm_mx8_test(A8, sA, W, bias, epi=5, variant=variant)
        assert torch.equal(got5, ref5), (rep, (got5.float() - ref5.float()).abs().max().item())
        q, s = E.gemm_mx8_test(A8, sA, W, bias, epi=4, variant=variant)
        assert torch.equal(s, ref4[1]) and torch.equal(q, ref4[0]), rep


def test_gemm_mx8_exact_integers(gpu):
    """Small integers are exact in e4m3 under any scale: C must equal the integer product."""
    M, N, K = 256, 512, 384
    g = torch.Generator().manual_seed(11)
    A = torch.randint(-3, 4, (M, K), generator=g).float()
    W = torch.randint(-3, 4, (N, K), generator=g).float()
    W[:, ::7] = 0
    A8, sA = E.quant_mx8_test(A.to(gpu))
    for variant in (1, 2):
        Cg = E.gemm_mx8_test(A8, sA, W.to(gpu), None, epi=0, variant=variant).cpu()
        assert torch.equal(Cg, A @ W.t()), variant


def test_gemm_mx8_epilogues(gpu):
    M, N, K = 515, 1024, 768
    A8, sA, W, bias, Ad, Wd = _quantized_operands(gpu, M, N, K, 21)
    c0 = E.gemm_mx8_test(A8, sA, W, bias, epi=0)
    c1 = E.gemm_mx8_test(A8, sA, W, bias, epi=1)
    ref = torch.from_numpy(Ad @ Wd.T).float() + bias.cpu()[None, :]
    gelu = ref * torch.sigmoid(1.702 * ref)
    assert ((c1.cpu() - gelu).abs().max() / gelu.abs().max()).item() < 1e-4
    # residual accumulate
    x0 = torch.randn(M, N, device=gpu)
    c2 = E.gemm_mx8_test(A8, sA, W, bias, epi=2, C=x0.clone())
    assert torch.allclose(c2, x0 + c0, rtol=0, atol=1e-5 * (x0 + c0).abs().max().item())
    # MX-fp8 outputs = quantization of the fp32 ones (same kernel arithmetic)
    for epi, base in ((3, c0), (4, c1)):
        q, s = E.gemm_mx8_test(A8, sA, W, bias, epi=epi)
        q_ref, s_ref = E.quant_mx8_test(base)
        assert torch.equal(s, s_ref) and torch.equal(q, q_ref), epi
    # bf16 store
    c5 = E.gemm_mx8_test(A8, sA, W, bias, epi=5)
    assert torch.equal(c5, c0.to(torch.bfloat16))


@pytest.mark.parametrize("M,N,K", [(257, 512, 512), (1000, 2304, 768), (333, 768, 3072),
                                   (12800, 2304, 768), (12800, 3072, 768), (25600, 3072, 768)])
def test_gemm_mx8_p32_tile(gpu, M, N, K):
    """MX variant 4 (gemm_p32mx.h: 32x32x64 scaled MFMA on the 4-stage 64-deep-k-step ring). Its
    fp32 sums group 64 products per instruction (variants 1-3: 128), so it is checked against
    the fp64 product of the same quantized operands (1e-4 of max|C|, the bar of the other
    tiles), and its own outputs against each other bit for bit: the bf16 store equals the
    rounding of its fp32 output, the MX-fp8 QuickGELU output the quantization of its fp32
    QuickGELU output (launch_quant_mx8), over repeated launches (race screen)."""
    A8, sA, W, bias, Ad, Wd = _quantized_operands(gpu, M, N, K, M + N + K + 2)
    c0 = E.gemm_mx8_test(A8, sA, W, bias, epi=0, variant=4)
    ref = Ad @ Wd.T + bias.cpu().numpy()[None, :]
    err = np.abs(c0.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err < 1e-4, err
    c1 = E.gemm_mx8_test(A8, sA, W, bias, epi=1, variant=4)
    gelu = torch.from_numpy(ref).float()
    gelu = gelu * torch.sigmoid(1.702 * gelu)
    assert ((c1.cpu() - gelu).abs().max() / gelu.abs().max()).item() < 1e-4
    c5 = E.gemm_mx8_test(A8, sA, W, bias, epi=5, variant=4)
    assert torch.equal(c5, c0.to(torch.bfloat16))
    q_ref, s_ref = E.quant_mx8_test(c1)
    for rep in range(3):
        q, s = E.gemm_mx8_test(A8, sA, W, bias, epi=4, variant=4)
        assert torch.equal(s, s_ref) and torch.equal(q, q_ref), rep
        assert torch.equal(E.gemm_mx8_test(A8, sA, W, bias, epi=5, variant=4), c5), rep
        assert torch.equal(E.gemm_mx8_test(A8, sA, W, bias, epi=0, variant=4), c0), rep


def test_gemm_mx8_p32_exact_integers(gpu):
    """Small integers are exact in e4m3 under any scale: variant 4's C equals the integer product
    (ragged M: the last 256-row tile is mostly rows past M, dropped by the store range check)."""
    M, N, K = 300, 512, 1024
    g = torch.Generator().manual_seed(12)
    A = torch.randint(-3, 4, (M, K), generator=g).float()
    W = torch.randint(-3, 4, (N, K), generator=g).float()
    W[:, ::5] = 0
    A8, sA = E.quant_mx8_test(A.to(gpu))
    Cg = E.gemm_mx8_test(A8, sA, W.to(gpu), None, epi=0, variant=4).cpu()
    assert torch.equal(Cg, A @ W.t())


# ---------------------------------------------------------------- end to end (config 5)
def _engine(cfg, dtype, sd, adapters, T, segs, gpu, B, tuning=None):
    eng = VisionEngine(cfg, gpu, dtype, max_batch=B, tuning=tuning)
    eng.load_state_dict(sd)
    eng.load_lora(adapters)
    eng.set_text_features(T.numpy(), segs)
    return eng


def _peaked_text(anchor: torch.Tensor, C_: int, seed: int, a: float = 0.3) -> torch.Tensor:
    """Unit rows with cos(row, anchor) ~ a: 100*cos logits ~ 30 like real CLIP prompt pairs
    (the 'peaked' case of test_gpu_parity.py)."""
    g = torch.Generator().manual_seed(seed)
    T = torch.nn.functional.normalize(torch.randn(C_, anchor.numel(), generator=g), dim=-1)
    return torch.nn.functional.normalize(a * anchor[None, :] + (1 - a * a) ** 0.5 * T, dim=-1)


def test_mxfp8_logits_within_config5_bar(gpu):
    """Config 5 bar: MX-fp8 logits within 2e-2 (of max|logit|, per image) of the bf16 engine,
    asserted at realistic (peaked) logit scale. Against random text rows (logits ~ +-5, the
    hardest case for a relative bar) the deviation is reported, not asserted: e4m3 keeps 3
    mantissa bits, so every MX-fp8 GEMM output carries ~3-5 % relative noise."""
    cfg = C.get_config("ViT-B/32")
    sd = synthetic_state_dict(cfg, 0)
    adapters = synthetic_adapters(cfg, rank=8)
    g = torch.Generator().manual_seed(1234)
    segs = [0, 40, 60, 359, 395, 425, 437]
    B = 64
    px = torch.randn(B, 3, 224, 224, generator=g).clamp_(-1.8, 2.2).to(gpu)
    held = torch.randn(8, 3, 224, 224, generator=g).clamp_(-1.8, 2.2).to(gpu)
    T_rand = torch.nn.functional.normalize(torch.randn(437, cfg.embed_dim, generator=g), dim=-1)
    e16 = _engine(cfg, "bf16", sd, adapters, T_rand, segs, gpu, B)
    e8 = _engine(cfg, "mxfp8", sd, adapters, T_rand, segs, gpu, B)
    try:
        f = e16.encode_image(held).cpu()
        anchor = torch.nn.functional.normalize(torch.nn.functional.normalize(f, dim=-1).mean(0), dim=0)
        out = {}
        for name, T in (("random", T_rand), ("peaked", _peaked_text(anchor, 437, 7))):
            e16.set_text_features(T.numpy(), segs)
            e8.set_text_features(T.numpy(), segs)
            r16, r8 = e16.classify(px), e8.classify(px)
            l16, l8 = r16.logits.cpu(), r8.logits.cpu()
            rel = ((l8 - l16).abs().amax(1) / l16.abs().amax(1)).max().item()
            agree = (r8.top_idx[:, :, 0] == r16.top_idx[:, :, 0]).float().mean().item()
            cos = torch.nn.functional.cosine_similarity(r8.emb.cpu(), r16.emb.cpu(), dim=-1).min().item()
            out[name] = rel
            print(f"mxfp8 vs bf16 [{name}]: max rel logit err {rel:.4g}, top-1 agreement {agree:.3f}, "
                  f"min emb cosine {cos:.6f}")
        assert out["peaked"] <= 2e-2, out
    finally:
        e16.close()
        e8.close()


@pytest.mark.parametrize("model,skip,resid16", [("ViT-B/32", "", "1"), ("ViT-B/32", "0,1,10,11", "0"),
                                               ("ViT-B/16", None, None)])
def test_mxfp8_forward_variants(gpu, model, skip, resid16):
    """The MX-fp8 forward's other block layouts: every block MX-fp8 (tuning mx8_skip="": the last
    block runs on all rows, its c_proj adds into x in the MX GEMM epilogue, no class-token tail),
    the fp32 read-modify-write residual adds (resid16=0, the pre-r02 path), and the
    default layout on ViT-B/16 (N = 197). Against the bf16 engine at CLIP logit scale:
    embeddings aligned and logits within the all-MX-fp8 figure of DESIGN.md 5.7 (2.0e-2) plus
    margin."""
    cfg = C.get_config(model)
    sd = synthetic_state_dict(cfg, 0)
    adapters = synthetic_adapters(cfg, rank=8)
    g = torch.Generator().manual_seed(77)
    segs = [0, 40, 60, 359, 395, 425, 437]
    B = 16
    px = torch.randn(B, 3, cfg.image_size, cfg.image_size, generator=g).clamp_(-1.8, 2.2).to(gpu)
    T0 = torch.nn.functional.normalize(torch.randn(437, cfg.embed_dim, generator=g), dim=-1)
    e16 = _engine(cfg, "bf16", sd, adapters, T0, segs, gpu, B)
    tun = {}
    if skip is not None:
        tun["mx8_skip"] = skip
    if resid16 is not None:
        tun["resid16"] = resid16
    e8 = _engine(cfg, "mxfp8", sd, adapters, T0, segs, gpu, B, tuning=tun)
    try:
        f16 = e16.encode_image(px).cpu()
        anchor = torch.nn.functional.normalize(torch.nn.functional.normalize(f16, dim=-1).mean(0), dim=0)
        T = _peaked_text(anchor, 437, 5)
        e16.set_text_features(T.numpy(), segs)
        e8.set_text_features(T.numpy(), segs)
        r16, r8 = e16.classify(px), e8.classify(px)
        l16, l8 = r16.logits.cpu(), r8.logits.cpu()
        rel = ((l8 - l16).abs().amax(1) / l16.abs().amax(1)).max().item()
        cos = torch.nn.functional.cosine_similarity(r8.emb.cpu(), r16.emb.cpu(), dim=-1).min().item()
        print(f"mxfp8 {model} [skip {skip!r}, resid16 {resid16}] vs bf16: max rel logit err {rel:.4g}, min emb cosine {cos:.6f}")
        # the shipped default layout (skip None) meets the config-5 bar; the alternative layouts
        # are held to the all-MX-fp8 figure of DESIGN.md 5.7 (2.0e-2) plus margin
        assert cos > 0.99 and rel <= (2e-2 if skip is None and resid16 is None else 3e-2), (rel, cos)
    finally:
        e16.close()
        e8.close()


def test_attention_q8_output_bit_identical(gpu):
    """The MX-fp8 forward's attention writes the out_proj operand (MX-fp8) in its epilogue
    (ViT-B/32, N = 50): embeddings and logits must equal those of the two-kernel path
    (16-bit attention output + launch_quant_mx8, tuning attn_q8=0) bit for bit."""
    cfg = C.get_config("ViT-B/32")
    sd = synthetic_state_dict(cfg, 0)
    adapters = synthetic_adapters(cfg, rank=8)
    g = torch.Generator().manual_seed(91)
    segs = [0, 40, 60, 359, 395, 425, 437]
    B = 24
    px = torch.randn(B, 3, 224, 224, generator=g).clamp_(-1.8, 2.2).to(gpu)
    T = torch.nn.functional.normalize(torch.randn(437, cfg.embed_dim, generator=g), dim=-1)
    fused = _engine(cfg, "mxfp8", sd, adapters, T, segs, gpu, B)
    split = _engine(cfg, "mxfp8", sd, adapters, T, segs, gpu, B, tuning={"attn_q8": 0})
    try:
        a, b = fused.classify(px), split.classify(px)
        assert torch.equal(a.emb, b.emb)
        assert torch.equal(a.logits, b.logits)
    finally:
        fused.close()
        split.close()


def test_fp16_residual_stream_within_config5_bar(gpu):
    """MX-fp8 forward with the fp16 residual stream (the default, tuning x16) and with the fp32
    one, both against the bf16 engine at CLIP logit scale. The two MX-fp8 forwards differ by
    ~1.5e-2 from each other (any perturbation flips e4m3 roundings of the GEMM operands: the same
    size as the MX-fp8 error itself), so the check is on the error against bf16: the fp16 stream
    stays within the 2e-2 bar and within 5e-3 of the fp32 stream's error."""
    cfg = C.get_config("ViT-B/32")
    sd = synthetic_state_dict(cfg, 0)
    adapters = synthetic_adapters(cfg, rank=8)
    g = torch.Generator().manual_seed(92)
    segs = [0, 40, 60, 359, 395, 425, 437]
    B = 64
    px = torch.randn(B, 3, 224, 224, generator=g).clamp_(-1.8, 2.2).to(gpu)
    held = torch.randn(8, 3, 224, 224, generator=g).clamp_(-1.8, 2.2).to(gpu)
    T0 = torch.nn.functional.normalize(torch.randn(437, cfg.embed_dim, generator=g), dim=-1)
    e16 = _engine(cfg, "bf16", sd, adapters, T0, segs, gpu, B)
    x16 = _engine(cfg, "mxfp8", sd, adapters, T0, segs, gpu, B)
    x32 = _engine(cfg, "mxfp8", sd, adapters, T0, segs, gpu, B, tuning={"x16": 0})
    try:
        f = e16.encode_image(held).cpu()
        anchor = torch.nn.functional.normalize(torch.nn.functional.normalize(f, dim=-1).mean(0), dim=0)
        T = _peaked_text(anchor, 437, 9)
        for e in (e16, x16, x32):
            e.set_text_features(T.numpy(), segs)
        ref = e16.classify(px).logits.cpu()
        la, lb = x16.classify(px).logits.cpu(), x32.classify(px).logits.cpu()
        err = lambda l: ((l - ref).abs().amax(1) / ref.abs().amax(1)).max().item()
        ea, eb = err(la), err(lb)
        print(f"MX-fp8 vs bf16, peaked: fp16 residual {ea:.4g}, fp32 residual {eb:.4g}")
        assert not torch.equal(la, lb)  # the fp16 stream is really in use
        assert ea <= 2e-2 and ea <= eb + 5e-3, (ea, eb)
    finally:
        e16.close()
        x16.close()
        x32.close()


def test_config5_bs512_as_benched(gpu):
    """BASELINE config 5 exactly as bench.py --dtype mxfp8 --batch 512 runs it: ViT-B/32 + merged
    LoRA r=8, 512 images in one classify, which takes the two-lane split (256 images per lane
    stream) and the shipped MX-fp8 tiles (mx8_variants default) and bf16 block masks. Text rows
    at CLIP logit scale, built as tests/golden/make_golden.py clip_scale_text builds them
    (normalise(0.3 f + 0.95 r), f = the oracle's fp32 features of 16 of the images). Asserted:
    every one of the 512 images within 2e-2 of the bf16 engine (BASELINE's bar), 4 sample rows
    from both lanes within 2e-2 of the CPU fp32 oracle, and the two-lane split bit-identical to
    one stream (main.py:440-448 batches the same way)."""
    from oracle import clip_ref
    cfg = C.get_config("ViT-B/32")
    sd = synthetic_state_dict(cfg, 0)
    adapters = synthetic_adapters(cfg, rank=8)
    g = torch.Generator().manual_seed(512)
    segs = [0, 40, 60, 359, 395, 425, 437]
    B = 512
    px = torch.randn(B, 3, 224, 224, generator=g).clamp_(-1.8, 2.2)
    ref_sd = dict(sd)
    for a in adapters:
        ref_sd[a.target] = clip_ref.merge_lora(sd[a.target], torch.from_numpy(a.A), torch.from_numpy(a.B), a.scaling)
    probe = [0, 255, 256, 511] + list(range(1, 13))  # both lanes' first / last images first
    with torch.no_grad():
        f_ref = clip_ref.encode_image(ref_sd, clip_ref.GEOMETRIES[cfg.name], px[probe])
    gen = torch.Generator().manual_seed(2024)
    fn = torch.nn.functional.normalize(f_ref, dim=-1).double()
    r = torch.nn.functional.normalize(torch.randn(437, cfg.embed_dim, generator=gen, dtype=torch.float64), dim=-1)
    T = 0.3 * fn[torch.arange(437) % fn.shape[0]] + 0.95 * r
    T = (T / T.norm(dim=-1, keepdim=True)).float()
    pxg = px.to(gpu)
    e16 = _engine(cfg, "bf16", sd, adapters, T, segs, gpu, B)
    e8 = _engine(cfg, "mxfp8", sd, adapters, T, segs, gpu, B)
    one = _engine(cfg, "mxfp8", sd, adapters, T, segs, gpu, B, tuning={"split_min": 0})
    try:
        l16 = e16.classify(pxg).logits.cpu()
        r8 = e8.classify(pxg)
        l8 = r8.logits.cpu()
        ro = one.classify(pxg)
        torch.cuda.synchronize()
        assert torch.equal(r8.logits, ro.logits) and torch.equal(r8.emb, ro.emb)
        rel = ((l8 - l16).abs().amax(1) / l16.abs().amax(1))
        _, lo, _, _, _ = clip_ref.head(f_ref[:4], T, segs)
        rel_o = ((l8[probe[:4]] - lo).abs().amax(1) / lo.abs().amax(1))
        print(f"config 5 bs 512 (split, shipped MX tiles): vs bf16 worst {rel.max():.4g} median "
              f"{rel.median():.4g}; vs oracle rows {probe[:4]}: {rel_o.max():.4g}; "
              f"max |logit| median {l16.abs().amax(1).median():.1f}")
        assert rel.max().item() <= 2e-2, rel.max().item()
        assert rel_o.max().item() <= 2e-2, rel_o.max().item()
    finally:
        e16.close()
        e8.close()
        one.close()


def test_mx8_fc_round_split_is_bit_identical(gpu):
    """The MX-fp8 c_fc whole-round row split (clipvit.hip gemm8, tuning mx8_split_tail=2; off by
    default: 256 images = 12,800 rows = 600 tiles of 256x256 = 2 rounds + 88; rows [0, 10752) on
    the persistent ping-pong, the rest on the 128x128 tile, both writing the blocked u8 and its
    blocked scales) against one launch on the ping-pong: logits and embeddings bit for bit."""
    cfg = C.get_config("ViT-B/32")
    sd = synthetic_state_dict(cfg, 0)
    adapters = synthetic_adapters(cfg, rank=8)
    segs = [0, 40, 60, 359, 395, 425, 437]
    g = torch.Generator().manual_seed(77)
    T = torch.nn.functional.normalize(torch.randn(437, cfg.embed_dim, generator=g), dim=-1)
    px = torch.randn(256, 3, 224, 224, generator=g).clamp_(-1.8, 2.2).to(gpu)
    split = _engine(cfg, "mxfp8", sd, adapters, T, segs, gpu, 256, tuning={"mx8_split_tail": 2})
    one = _engine(cfg, "mxfp8", sd, adapters, T, segs, gpu, 256)
    try:
        a, b = split.classify(px), one.classify(px)
        torch.cuda.synchronize()
        assert torch.equal(a.emb, b.emb) and torch.equal(a.logits, b.logits)
    finally:
        split.close()
        one.close()
