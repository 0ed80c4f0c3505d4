"""Per-kernel parity on the GPU, through the C ABI test entry points.

GEMM: fp32 torch reference of the same op on the 16-bit-rounded operands (tolerance from
fp32-accumulation order only: 2e-3 relative to max|C|). Attention: the oracle's fp32
attention on the same 16-bit q/k/v; P is rounded to 16 bit before P.V (flash-style), so the
bound is 1e-2 of max|O| for bf16 and 3e-3 for fp16.
"""
import math

import pytest
import torch

from interior_amd import engine as E

pytestmark = pytest.mark.gpu


def _ref_gemm(A, W, bias, epi, C0=None):
    ref = A.float() @ W.to(A.dtype).float().t()
    if bias is not None:
        ref = ref + bias
    if epi == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    if epi == 2:
        ref = ref + C0
    return ref


# variant = 100 * xcd_partition + tile kernel (gemm.hip launch_t); 2xx = 4x2 XCD tile partition,
# 34xx / 35xx = column-group-major 1-D remap with 2 / 3 N-groups (tile_of_block).
# The shipped tiles: 1-3 shape fallback, 8 / 80 256x256, 81 128x128, 22 / 82 160x128,
# 98 240x256 (12 waves), 90 64x64 (class-token tail), 62 the persistent 256x256 ping-pong tile
# (gemm_pp.hip; 72 the 32-deep-k-step persistent tile of
# gemm_p32.h; 74 the same with non-temporal stores; 75 on a balanced grid; 77 its 320 x 256 form on a balanced
# grid; 79 its 192 x 256 form on a balanced grid); + 10000 = W in the 16-row blocked layout (GemmArgs.blk_w, tuning w_blocked);
# 2xx = the production XCD partition.
VARIANTS = [1, 2, 3, 8, 22, 62, 72, 74, 75, 77, 79, 81, 82, 90, 98, 208, 222, 282, 298, 3408, 3462, 3472,
            3474, 3477, 3479, 10008, 10022, 10062, 10072, 10077, 10079, 10081, 10082, 10090, 10098, 13462, 13472,
            13477, 13479]
N128 = (1, 2, 22, 81, 82)
N256 = (3, 8, 62, 72, 74, 75, 77, 79, 98)
STAGED = (62, 72, 74, 75, 77, 79, 81, 82, 98)  # 16-bit outputs only (rounded to 16 bits)


def _tol(variant, dtype):
    """fp32 outputs: accumulation order only. 16-bit outputs add one rounding of the output:
    2^-8 relative for bf16 near max|C| (an order flip can cost a full ulp)."""
    if variant % 100 in STAGED and dtype == torch.bfloat16:
        return 8e-3
    return 2e-3


def _skip(variant, N, K):
    v = variant % 100
    if (v in N128 and N % 128) or (v in N256 and N % 256):
        return "tile does not divide N"
    if v in (62, 63) and K % 128:
        return "ping-pong tile: K in pairs of 64-deep k-tiles"
    if v in (72, 74, 75, 77, 79) and (K % 128 or K < 256):
        return "32-deep-k-step tile: K a multiple of 128, >= 256"
    return None


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("M,N,K", [(12800, 768, 768), (1000, 2304, 768), (333, 3072, 768),
                                   (700, 768, 3072), (64, 256, 64)])
def test_gemm_shapes(gpu, dtype, variant, M, N, K):
    why = _skip(variant, N, K)
    if why:
        pytest.skip(why)
    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    A = torch.randn(M, K, device=gpu, generator=g).to(dtype)
    W = torch.randn(N, K, device=gpu, generator=g) * 0.05
    bias = torch.randn(N, device=gpu, generator=g)
    C = E.gemm_test(A, W, bias, epi=0, variant=variant)
    ref = _ref_gemm(A, W, bias, 0)
    err = (C - ref).abs().max().item() / ref.abs().max().item()
    assert err < _tol(variant, dtype), err


@pytest.mark.parametrize("variant", STAGED + (8, 22, 10072, 10077, 10079, 10081, 10098))
@pytest.mark.parametrize("epi", [10, 11])
def test_gemm_staged_16bit_epilogue(gpu, variant, epi):
    """16-bit STORE / GELU epilogues on ragged M (last tile partial): LDS-staged row-contiguous
    (81, 82, 98) and direct from the accumulators (8, 22, 62, 72-77)."""
    dtype = torch.float16
    M, N, K = 1000, 2304, 768
    if N % (256 if variant in N256 else 128):
        pytest.skip("tile does not divide N")
    g = torch.Generator(device=gpu).manual_seed(11)
    A = torch.randn(M, K, device=gpu, generator=g).to(dtype)
    W = torch.randn(N, K, device=gpu, generator=g) * 0.05
    bias = torch.randn(N, device=gpu, generator=g)
    C = E.gemm_test(A, W, bias, epi=epi, variant=variant)
    ref = _ref_gemm(A, W, bias, epi - 10)
    err = (C - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-3, err


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("variant,M,N,K,S", [(90, 256, 768, 3072, 8), (90, 67, 3072, 768, 4),
                                             (90, 9, 768, 768, 4), (90, 256, 1024, 1024, 4),
                                             (8, 300, 512, 1024, 2), (82, 333, 768, 1536, 3)])
def test_gemm_split_k(gpu, dtype, variant, M, N, K, S):
    """Split-K (the class-token tail's GEMMs): slice z of grid.y writes the fp32 partial of
    k in [z K/S, (z + 1) K/S) to C[z]; each partial is checked against its own K slice, so a
    slice offset error cannot cancel in the sum. Ragged M included."""
    g = torch.Generator(device=gpu).manual_seed(M + N + K + S)
    A = torch.randn(M, K, device=gpu, generator=g).to(dtype)
    W = torch.randn(N, K, device=gpu, generator=g) * 0.05
    C = torch.full((S * M, N), float("nan"), device=gpu)
    C = E.gemm_test(A, W, None, epi=20 + S, variant=variant, C=C).reshape(S, M, N)
    ks = K // S
    for z in range(S):
        ref = _ref_gemm(A[:, z * ks:(z + 1) * ks], W[:, z * ks:(z + 1) * ks], None, 0)
        err = (C[z] - ref).abs().max().item() / ref.abs().max().item()
        assert err < 2e-3, (z, err)


def test_gemm_split_k_refuses_bad_slices(gpu):
    """K not divisible into 64-deep slices, or a non-pipelined tile: the library refuses."""
    A = torch.zeros(64, 768, device=gpu, dtype=torch.float16)
    W = torch.zeros(64, 768, device=gpu)
    C = torch.zeros(8 * 64, 64, device=gpu)
    with pytest.raises(Exception):
        E.gemm_test(A, W, None, epi=20 + 8, variant=90, C=C)  # 768 / 8 = 96: not a multiple of 64
    with pytest.raises(Exception):
        E.gemm_test(A, W, None, epi=20 + 4, variant=1, C=C)


@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_epilogues(gpu, epi):
    dtype = torch.bfloat16
    M, N, K = 515, 1024, 512
    g = torch.Generator(device=gpu).manual_seed(7)
    A = torch.randn(M, K, device=gpu, generator=g).to(dtype)
    W = torch.randn(N, K, device=gpu, generator=g) * 0.05
    bias = torch.randn(N, device=gpu, generator=g)
    C0 = torch.randn(M, N, device=gpu, generator=g)
    C = E.gemm_test(A, W, bias, epi=epi, variant=0, C=C0.clone())
    ref = _ref_gemm(A, W, bias, epi, C0)
    err = (C - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-3, err


def test_gemm_asymmetric_identity(gpu):
    """A = I, asymmetric W: catches any row/column or permutation mix-up in the epilogue."""
    K = N = 256
    A = torch.eye(K, device=gpu).to(torch.bfloat16)
    W = (torch.arange(N * K, device=gpu, dtype=torch.float32).reshape(N, K) % 251) / 8.0
    for variant in VARIANTS:
        C = E.gemm_test(A, W, None, epi=0, variant=variant)
        assert torch.equal(C, W.to(torch.bfloat16).float().t()), variant


def _ref_attention(qkv, B, N, H, causal=False):
    D = H * 64
    x = qkv.float().reshape(B, N, 3, H, 64)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(64)
    if causal:
        s = s + torch.full((N, N), float("-inf"), device=s.device).triu(1)
    o = s.softmax(-1) @ v
    return o.transpose(1, 2).reshape(B * N, D)


@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 1e-2), (torch.float16, 3e-3)])
@pytest.mark.parametrize("B,N,H", [(3, 50, 12), (2, 197, 12), (1, 577, 16), (2, 1, 12), (1, 65, 12),
                                   (2, 130, 12), (1, 300, 16)])
def test_attention(gpu, dtype, tol, B, N, H):
    g = torch.Generator(device=gpu).manual_seed(B * N * H)
    qkv = (torch.randn(B * N, 3 * H * 64, device=gpu, generator=g) * 1.5).to(dtype)
    out = E.attention_test(qkv, B, N, H)
    ref = _ref_attention(qkv, B, N, H)
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < tol, err


@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 1e-2), (torch.float16, 3e-3)])
@pytest.mark.parametrize("B,N,H", [(3, 77, 8), (2, 1, 8), (1, 64, 8), (2, 65, 8), (1, 200, 12)])
def test_attention_causal(gpu, dtype, tol, B, N, H):
    """The text tower's causal attention (CLIP.build_attention_mask: -inf above the diagonal)
    against the fp32 reference, including blocks past the last query and single-token rows."""
    g = torch.Generator(device=gpu).manual_seed(B * N * H + 1)
    qkv = (torch.randn(B * N, 3 * H * 64, device=gpu, generator=g) * 1.5).to(dtype)
    out = E.attention_test(qkv, B, N, H, causal=True)
    ref = _ref_attention(qkv, B, N, H, causal=True)
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < tol, err


def test_attention_spiky_scores(gpu):
    """A key far above the rest of its block forces the online-softmax rescale across
    key blocks (N = 197 -> 4 key blocks): the late block's max must rescale earlier blocks."""
    B, N, H = 1, 197, 12
    g = torch.Generator(device=gpu).manual_seed(3)
    qkv = torch.randn(B * N, 3 * H * 64, device=gpu, generator=g)
    qkv[150, H * 64: 2 * H * 64] *= 6.0   # one large key in the third block
    qkv = qkv.to(torch.float16)
    out = E.attention_test(qkv, B, N, H)
    ref = _ref_attention(qkv, B, N, H)
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 3e-3, err


@pytest.mark.parametrize("B,N,H,causal", [(2, 77, 8, True), (2, 197, 12, False), (1, 577, 16, False),
                                          (2, 130, 12, False), (1, 65, 12, False), (3, 50, 12, False)])
def test_attention_tail_rows_never_read(gpu, B, N, H, causal):
    """qkv is a view into a larger buffer whose rows after B*N are NaN. Key rows past N in the
    last key block must never be fetched (a range check that misses an SGPR block
    offset would read them), so the output stays finite and matches the reference."""
    g = torch.Generator(device=gpu).manual_seed(B * N + H)
    big = torch.full((B * N + 128, 3 * H * 64), float("nan"), device=gpu, dtype=torch.float16)
    big[:B * N] = (torch.randn(B * N, 3 * H * 64, device=gpu, generator=g) * 1.5).half()
    qkv = big[:B * N]
    out = E.attention_test(qkv, B, N, H, causal=causal)
    assert torch.isfinite(out).all()
    ref = _ref_attention(qkv, B, N, H, causal=causal)
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 3e-3, err


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("B,N,H,persist", [(3, 50, 12, 1), (256, 50, 12, 2), (256, 50, 12, 1), (7, 64, 12, 2),
                                           (5, 1, 12, 1), (300, 33, 12, 3), (1, 50, 2, 4)])
def test_attention_persistent_bit_identical(gpu, dtype, B, N, H, persist):
    """The persistent one-key-block attention (tuning attn_persist: each workgroup walks several
    (image, head) units, prefetching the next unit's K/V / Q while computing the current one) runs
    attention_v2's per-unit arithmetic: its output equals attention_v2's bit for bit, for fewer
    units than workgroups, several units per workgroup and ragged N; repeated launches agree, and
    NaN rows past the last image are never read."""
    g = torch.Generator(device=gpu).manual_seed(B * N + H + persist)
    big = torch.full((B * N + 128, 3 * H * 64), float("nan"), device=gpu, dtype=dtype)
    big[:B * N] = (torch.randn(B * N, 3 * H * 64, device=gpu, generator=g) * 1.5).to(dtype)
    qkv = big[:B * N]
    ref = E.attention_test(qkv, B, N, H)
    for rep in range(3):
        out = E.attention_test(qkv, B, N, H, persist=persist)
        assert torch.equal(out, ref), (rep, (out.float() - ref.float()).abs().max().item())


@pytest.mark.parametrize("M,N,K", [(12800, 3072, 768), (10752, 3072, 768), (1000, 2304, 768), (333, 768, 3072), (12800, 768, 3072),
                                   (36928 // 4, 4096, 1024)])
def test_ping_pong_race_screen(gpu, M, N, K):
    """The persistent ping-pong GEMM (62; + 10000 with the blocked weight copy) hands LDS stages between waves by counted vmcnt and
    barriers only. Every accumulator sees the same k order as the 2-phase 256x256 tile (v8), so
    the outputs must equal v8's bit for bit on every one of many repeated launches: a read that
    overtook its DMA (or a refill that overtook a read) would show as a differing tile."""
    g = torch.Generator(device=gpu).manual_seed(M + N)
    A = torch.randn(M, K, device=gpu, generator=g).to(torch.float16)
    W = torch.randn(N, K, device=gpu, generator=g) * 0.05
    bias = torch.randn(N, device=gpu, generator=g)
    for epi in (10, 11):  # 16-bit store / QuickGELU
        ref = E.gemm_test(A, W, bias, epi=epi, variant=8)
        for variant in (62, 3462, 10062, 13462):  # + 10000: blocked weight copy
            for _ in range(6):
                C = E.gemm_test(A, W, bias, epi=epi, variant=variant)
                assert torch.equal(C, ref), (variant, epi, (C - ref).abs().max().item())


@pytest.mark.parametrize("M,N,K", [(12800, 3072, 768), (10752, 3072, 768), (1000, 2304, 768), (333, 768, 3072), (12800, 768, 3072),
                                   (36928 // 4, 4096, 1024), (50432, 2304, 768)])
def test_p32_race_screen(gpu, M, N, K):
    """The 32-deep-k-step persistent tiles (72 / 74 non-temporal / 75 on the balanced grid / 77 its 320 x 256 form; the large-M roles' and the B/32
    c_fc main launch's default since r05, with the blocked weight copy: + 10000) hand their four
    LDS stages between the two wave groups by counted vmcnt and barriers only. Their arithmetic is
    v8's (accumulate from 0, then + bias, QuickGELU), so the outputs must equal v8's bit for bit
    on every one of many repeated launches: a read that overtook its DMA (or a refill that
    overtook a read) would show as a differing tile, and a different bit pattern would make the
    tile choice (per shape, per lane split) change results."""
    g = torch.Generator(device=gpu).manual_seed(M + N + 1)
    A = torch.randn(M, K, device=gpu, generator=g).to(torch.float16)
    W = torch.randn(N, K, device=gpu, generator=g) * 0.05
    bias = torch.randn(N, device=gpu, generator=g)
    for epi in (10, 11):  # 16-bit store / QuickGELU
        ref = E.gemm_test(A, W, bias, epi=epi, variant=8)
        for variant in (72, 3472, 10072, 13472, 74, 13474, 10075, 77, 3477, 10077, 13477, 79, 10079, 13479):
            for _ in range(4):
                C = E.gemm_test(A, W, bias, epi=epi, variant=variant)
                assert torch.equal(C, ref), (variant, epi, (C - ref).abs().max().item())


def test_residual_x24_round_trip(gpu):
    """The 24-bit residual stream (the 16-bit forward's x between the LayerNorm kernels): the
    upper 16 bits of each fp32 value plus the next 8, rounded to nearest at bit 8 (a carry into
    the exponent rounds up to the next binade). The device round trip equals that rule bit for
    bit and stays within 2^-16 relative."""
    g = torch.Generator().manual_seed(24)
    x = torch.cat([torch.randn(4096, generator=g) * 10.0 ** torch.randint(-6, 6, (4096,), generator=g),
                   torch.tensor([0.0, -0.0, 1.0, -1.0, 2.0 ** -20, 65504.0, 1e30, -3.0e-38]),
                   # values on and beside the rounding boundary of bit 8
                   torch.tensor([1.0, 1.0]).view(torch.int32).add(
                       torch.tensor([0x7F, 0x80], dtype=torch.int32)).view(torch.float32),
                   torch.tensor([1.0, -1.0]).view(torch.int32).add(
                       torch.tensor([0xFFFF80, 0xFFFF7F], dtype=torch.int32)).view(torch.float32)])
    assert torch.isfinite(x).all()
    x = x[: x.numel() // 4 * 4]
    back = E.residual_x24_test(x.to(gpu)).cpu()
    bits = x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    ref = (((bits + 0x80) & 0xFFFFFF00) & 0xFFFFFFFF).to(torch.int64)
    ref = torch.where(ref >= 2 ** 31, ref - 2 ** 32, ref).to(torch.int32).view(torch.float32)
    assert torch.equal(back.view(torch.int32), ref.view(torch.int32))
    nz = x != 0
    rel = ((back - x).abs()[nz] / x.abs()[nz]).max().item()
    assert rel <= 2.0 ** -16, rel


@pytest.mark.parametrize("variant", [8, 22, 62, 72, 75, 77, 79, 81, 82, 98, 298, 3475, 3477, 3479])
@pytest.mark.parametrize("M,N,K", [(1000, 2304, 768), (12800, 3072, 768)])
def test_blocked_a_is_bit_identical(gpu, variant, M, N, K):
    """A (the LayerNorm output h that QKV / c_fc read) in the 16-row blocked layout (+ 20000; with
    the blocked weight copy + 30000) moves bytes only: every tile stages the same k-slices into
    the same LDS image, so the 16-bit STORE / QuickGELU outputs equal the row-major run's bit for
    bit, ragged M included."""
    if N % (256 if variant % 100 in N256 else 128):
        pytest.skip("tile does not divide N")
    g = torch.Generator(device=gpu).manual_seed(M + K + 7)
    A = torch.randn(M, K, device=gpu, generator=g).to(torch.float16)
    W = torch.randn(N, K, device=gpu, generator=g) * 0.05
    bias = torch.randn(N, device=gpu, generator=g)
    for epi in (10, 11):
        ref = E.gemm_test(A, W, bias, epi=epi, variant=variant)
        for v in (20000 + variant, 30000 + variant):
            C = E.gemm_test(A, W, bias, epi=epi, variant=v)
            assert torch.equal(C, ref), (v, epi, (C - ref).abs().max().item())
