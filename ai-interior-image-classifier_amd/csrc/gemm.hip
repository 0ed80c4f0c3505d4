// MFMA GEMM for every dense contraction of the CLIP ViT encoder (gfx950, wave64).
//
//   C[M, N] = A[M, K] @ W[N, K]^T (+ bias) with a fused epilogue
//
// A = token activations (row-major, K contiguous), W = nn.Linear weight [out, in] as stored
// by OpenAI CLIP (attn.in_proj_weight, attn.out_proj.weight, mlp.c_fc.weight,
// mlp.c_proj.weight; conv1.weight viewed as [width, 3*p*p]).  Both operands are K-major, so
// every MFMA fragment is one 16-byte LDS read.
//
// Design:
//  * block tile BM x BN x 64, waves arranged WM x WN, each wave TM x TN = (BM/WM) x (BN/WN);
//  * global -> LDS by global_load_lds_dwordx4 (no VGPR staging), two LDS buffers, next tile's
//    loads issued before the current tile's MFMAs;
//  * LDS rows are 128 B (64 x 16-bit); 16-B chunk c of row r lives at chunk c ^ (r & 7) — the
//    swizzle is applied to the per-lane global SOURCE address (glds writes lane-linearly) and to
//    the ds_read address, which makes every ds_read_b128 wave-instruction conflict-free;
//  * swapped operands: MFMA A-operand = weight rows, B-operand = token rows, so the 16x16
//    accumulator holds C^T: lane (j = lane&15, g = lane>>4) owns token j and 4 features.
//    W is packed with its rows permuted inside every 64-row group (launch_pack_weight) so that
//    over four consecutive 16-row subtiles a lane owns 16 CONTIGUOUS output features -> 32-B
//    (16-bit) or 64-B (fp32) vector stores in the epilogue, no shuffles;
//  * v_mfma_f32_16x16x32_{bf16,f16}, fp32 accumulation; epilogue adds bias, QuickGELU
//    (x * sigmoid(1.702 x), CLIP's activation) or the fp32 residual add;
//  * bijective XCD-aware block remap: consecutive logical tiles (same A panel) share an XCD L2.
#include <algorithm>
#include <type_traits>
#include "common.h"

namespace clipvit {

template <typename T, int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(64 * WM* WN) void gemm_nt_kernel(GemmArgs a) {
    typedef typename T::vec8 vec8;
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    static_assert(TN % 64 == 0, "wave N-tile must be a multiple of 64 (packed groups)");
    static_assert(TM % 16 == 0, "wave M-tile must be a multiple of 16");
    constexpr int A_BYTES = BM * 128, W_BYTES = BN * 128;
    static_assert(A_BYTES % (NT * 16) == 0 && W_BYTES % (NT * 16) == 0, "staging rounds");
    constexpr int STAGE = A_BYTES + W_BYTES;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;

    const int nN = a.N / BN;
    const int nwg = gridDim.x;
    int bid = blockIdx.x;
    {  // bijective XCD remap: blocks b, b+8, ... (one XCD) take a contiguous logical range
        const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    }
    const int m0 = (bid / nN) * BM, n0 = (bid % nN) * BN;

    const unsigned char* Ab = (const unsigned char*)a.A;
    const unsigned char* Wb = (const unsigned char*)a.W;
    const size_t ldb = (size_t)a.K * 2;  // row stride in bytes (A and W)
    const int mlast = a.M - 1;

    auto stage = [&](int buf, int kt) {
        unsigned char* sA = smem + buf * STAGE;
        unsigned char* sW = sA + A_BYTES;
        const size_t kofs = (size_t)kt * 128;
#pragma unroll
        for (int r = 0; r < A_BYTES / (NT * 16); ++r) {
            const int p = r * NT * 16 + tid * 16;
            const int row = p >> 7, c = ((p >> 4) & 7) ^ (row & 7);
            const int grow = min(m0 + row, mlast);
            glds16(Ab + (size_t)grow * ldb + kofs + c * 16, sA + r * NT * 16 + wave * 1024);
        }
#pragma unroll
        for (int r = 0; r < W_BYTES / (NT * 16); ++r) {
            const int p = r * NT * 16 + tid * 16;
            const int row = p >> 7, c = ((p >> 4) & 7) ^ (row & 7);
            glds16(Wb + (size_t)(n0 + row) * ldb + kofs + c * 16, sW + r * NT * 16 + wave * 1024);
        }
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = a.K >> 6;
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int lrow = lane & 15, lsw = lane & 7;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
        const unsigned char* sA = smem + cur * STAGE;
        const unsigned char* sW = sA + A_BYTES;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int c = ((s << 2) | (lane >> 4)) ^ lsw;
            vec8 af[FM], wf[FN];
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
                af[fm] = *(const vec8*)(sA + (wm * TM + fm * 16 + lrow) * 128 + (c << 4));
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
                wf[fn] = *(const vec8*)(sW + (wn * TN + fn * 16 + lrow) * 128 + (c << 4));
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
#pragma unroll
                for (int fm = 0; fm < FM; ++fm) acc[fn][fm] = T::mfma16(wf[fn], af[fm], acc[fn][fm]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---- epilogue: lane owns token m and features n .. n+15 of each 64-feature group ----
    const int g = lane >> 4;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
        const int m = m0 + wm * TM + fm * 16 + lrow;
        if (m >= a.M) continue;
#pragma unroll
        for (int q = 0; q < FN / 4; ++q) {
            const int n = n0 + wn * TN + q * 64 + 16 * g;
            float v[16];
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[4 * f + r] = acc[4 * q + f][fm][r];
            if constexpr (EPI != EPI_PATCH) {
                if (a.bias) {
                    const float4* b4 = (const float4*)(a.bias + n);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float4 bb = b4[i];
                        v[4 * i] += bb.x; v[4 * i + 1] += bb.y; v[4 * i + 2] += bb.z; v[4 * i + 3] += bb.w;
                    }
                }
            }
            if constexpr (EPI == EPI_GELU || EPI == EPI_F32GELU) {
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = quick_gelu(v[i]);
            }
            if constexpr (EPI == EPI_STORE || EPI == EPI_GELU) {
                uint4* dst = (uint4*)((u16*)a.C + (size_t)m * a.ldc + n);
                dst[0] = make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]),
                                    pack2<T>(v[6], v[7]));
                dst[1] = make_uint4(pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]),
                                    pack2<T>(v[12], v[13]), pack2<T>(v[14], v[15]));
            } else if constexpr (EPI == EPI_RESID) {
                float4* dst = (float4*)((float*)a.C + (size_t)m * a.ldc + n);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float4 o = dst[i];
                    o.x += v[4 * i]; o.y += v[4 * i + 1]; o.z += v[4 * i + 2]; o.w += v[4 * i + 3];
                    dst[i] = o;
                }
            } else {
                size_t row = (size_t)m;
                if constexpr (EPI == EPI_PATCH)
                    row = (size_t)(m / a.patch_g2) * a.patch_ntok + 1 + (m % a.patch_g2);
                float4* dst = (float4*)((float*)a.C + row * a.ldc + n);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    dst[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Pipelined variant: an NS-stage LDS ring (BK = 64) filled by global_load_lds; loads of up to
// NS-1 tiles stay in flight ACROSS barriers (raw s_barrier + hand-counted vmcnt, never
// __syncthreads(), which would drain vmcnt to 0); fragments for the next 32-deep k-substep
// are read from LDS while the current substep's MFMAs run, and the barrier that hands over
// tile kt+1 sits between the last ds_read of tile kt and its last MFMAs.
// Wait until the awaited tile's loads have landed, given r = number of tiles (LPT loads each)
// issued after it that may stay in flight (0 <= r <= NS - 2).
template <int LPT, int NS>
__device__ __forceinline__ void wait_tile(int r) {
    if constexpr (NS - 2 >= 2) {
        if (r >= 2) { vm_wait<2 * LPT>(); return; }
    }
    if constexpr (NS - 2 >= 1) {
        if (r >= 1) { vm_wait<LPT>(); return; }
    }
    vm_wait<0>();
}

// Implicit-GEMM patch embedding (PIMPL = patch size P > 0): the A operand is the 16-bit NCHW
// pixel tensor itself. Row m of A = patch (image b, py, px); the patch's k order is
// k = c * (P * PP) + r * PP + j (PP = P rounded up to a multiple of 8), so every 8-element
// (16-byte) LDS chunk is 8 consecutive pixels of ONE pixel row. Pixel rows hold G * PP pixels
// (a.patch_Rw): for P = 14 the input is first copied with every 14-pixel patch row padded to 16
// (launch_cast_pixels_padded; the packed conv weight is zero at j = 14, 15), for P = 16 / 32 the
// pixels are used as given. Each staging piece is a global_load_lds from
// pix + patch_base(m) + patch_koff(k): the patch tile goes straight from the image into LDS,
// with no im2col buffer.
template <int P>
__device__ __forceinline__ int patch_koff(int kq, int R, int Rw) {
    constexpr int PP = (P + 7) / 8 * 8, CH = P * PP;
    if (kq >= 3 * CH) return 0;  // K padding: any in-bounds address (the weights there are zero)
    const int c = kq / CH, rem = kq - c * CH, r = rem / PP, j0 = rem - r * PP;
    return (c * R + r) * Rw + j0;
}

// v[i] += bias[i] for the lane's 16 contiguous features (bias staged in LDS; zero when absent)
__device__ __forceinline__ void colv_add(float (&v)[16], const float* bias) {
    const float4* b4 = (const float4*)bias;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float4 bb = b4[i];
        v[4 * i] += bb.x; v[4 * i + 1] += bb.y; v[4 * i + 2] += bb.z; v[4 * i + 3] += bb.w;
    }
}

// v[i] = rstd (v[i] - mu s[i]) + b'[i] for the lane's 16 contiguous features (EPI_LNF*)
__device__ __forceinline__ void lnf_apply(float (&v)[16], const float* __restrict__ s, const float* __restrict__ bp,
                                          float mu, float rstd) {
    const float4* s4 = (const float4*)s;
    const float4* b4 = (const float4*)bp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float4 ss = s4[i], bb = b4[i];
        v[4 * i] = rstd * (v[4 * i] - mu * ss.x) + bb.x;
        v[4 * i + 1] = rstd * (v[4 * i + 1] - mu * ss.y) + bb.y;
        v[4 * i + 2] = rstd * (v[4 * i + 2] - mu * ss.z) + bb.z;
        v[4 * i + 3] = rstd * (v[4 * i + 3] - mu * ss.w) + bb.w;
    }
}

// EPI_RES_STATS (residual producers out_proj / c_proj): x += acc + bias (fp32, the same additions
// as EPI_RESID; x read and written as fp32 or, with a.x24_plane, as the 24-bit planes: the sum is
// rounded to 24 bits only where it is stored, as launch_add_layernorm_deferred does), x16 = x
// (16-bit, of the fp32 sum), and per row the (mean, M2) of the fp32 sum over each 128-column group = two
// adjacent 64-column waves (TN == 64): the 64-column sums are shuffle-reduced over the 4 lanes of
// a row, exchanged with the partner wave through LDS, then the squared deviations from the
// group mean the same way (two-pass, no cancellation).
template <typename T, int FM, int FN, int TM, int TN, int WN, bool PREX>
__device__ __forceinline__ void res_stats_epilogue(const GemmArgs& a, f32x4 (&acc)[FN][FM],
                                                   const float4 (&xpre)[PREX ? FM : 1][4],
                                                   const float* bias, unsigned char* smem,
                                                   int m0, int n0, int wm, int wn, int lane) {
    static_assert(TN == 64 && FN == 4 && WN % 2 == 0, "statistics groups = two 64-wide waves");
    const int lrow = lane & 15, g = lane >> 4;
    float* red = (float*)smem;  // [waves][FM][16] partial sums, then the same for M2
    const int wave = wm * WN + wn, partner = wm * WN + (wn ^ 1);
    constexpr int NW = 64 * FM * 16;  // floats per exchange region (64 waves max)
    __builtin_amdgcn_s_barrier();      // every wave is done reading the LDS ring
    float sum[FM];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
        const int m = m0 + wm * TM + fm * 16 + lrow;
        const int n = n0 + wn * TN + 16 * g;
        const size_t xi = (size_t)min(m, a.M - 1) * a.ldc + n;  // x element index (fp32 or 24-bit planes)
        float* xr = (float*)a.C + xi;
        unsigned char* const xb = (unsigned char*)a.C;
        const float4* b4 = (const float4*)bias;
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 bb = b4[i];
            const float4 xo = PREX ? xpre[PREX ? fm : 0][i]
                                   : (a.x24_plane ? x24_load(xb, a.x24_plane, xi + 4 * i) : ((const float4*)xr)[i]);
            f32x4& c = acc[i][fm];
            c[0] = xo.x + (c[0] + bb.x);
            c[1] = xo.y + (c[1] + bb.y);
            c[2] = xo.z + (c[2] + bb.z);
            c[3] = xo.w + (c[3] + bb.w);
            s += (c[0] + c[1]) + (c[2] + c[3]);
        }
        if (m < a.M) {
            unsigned char* hr = (unsigned char*)a.C2 + ((size_t)m * a.ldc + n) * 2;
            if (a.x24_plane) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    x24_store(xb, a.x24_plane, xi + 4 * i, make_float4(acc[i][fm][0], acc[i][fm][1], acc[i][fm][2], acc[i][fm][3]));
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    ((float4*)xr)[i] = make_float4(acc[i][fm][0], acc[i][fm][1], acc[i][fm][2], acc[i][fm][3]);
            }
            *(uint4*)hr = make_uint4(pack2<T>(acc[0][fm][0], acc[0][fm][1]), pack2<T>(acc[0][fm][2], acc[0][fm][3]),
                                     pack2<T>(acc[1][fm][0], acc[1][fm][1]), pack2<T>(acc[1][fm][2], acc[1][fm][3]));
            *(uint4*)(hr + 16) = make_uint4(pack2<T>(acc[2][fm][0], acc[2][fm][1]), pack2<T>(acc[2][fm][2], acc[2][fm][3]),
                                            pack2<T>(acc[3][fm][0], acc[3][fm][1]), pack2<T>(acc[3][fm][2], acc[3][fm][3]));
        }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        sum[fm] = s;
        if (g == 0) red[(wave * FM + fm) * 16 + lrow] = s;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    float mean[FM];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
        const float ps = red[(partner * FM + fm) * 16 + lrow];
        mean[fm] = ((wn & 1) ? (ps + sum[fm]) : (sum[fm] + ps)) * (1.0f / 128.f);  // same order in both waves
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float d = acc[i][fm][r] - mean[fm];
                q += d * d;
            }
        q += __shfl_xor(q, 16, 64);
        q += __shfl_xor(q, 32, 64);
        sum[fm] = q;
        if (g == 0) red[NW + (wave * FM + fm) * 16 + lrow] = q;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if ((wn & 1) == 0 && g == 0) {
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
            const int m = m0 + wm * TM + fm * 16 + lrow;
            if (m < a.M) {
                const float m2 = sum[fm] + red[NW + (partner * FM + fm) * 16 + lrow];
                a.st_out[(size_t)m * a.np + (n0 + wn * TN) / 128] = make_float2(mean[fm], m2);
            }
        }
    }
}

// SM = 3: 16-bit outputs are staged through LDS and stored as whole rows (see the epilogue).
// 16-bit C stores of the pipelined tiles' epilogues: cache policy PIPE_AUX_ST (0 = plain global
// stores; otherwise buffer stores over C with those policy bits; default sc0 sc1, common.h
// GEMM_ST_AUX). r06 same box, B/32 bs 256: out_proj 0.245 -> 0.225 ms, c_proj 0.665 -> 0.658 ms
// per forward, +1.1 % against plain stores; the patch GEMM's fp32 rows stay plain (sc0 sc1 there:
// patch family 0.12 -> 0.15 ms; profiles/r06/store_policy_ab.txt)
#ifndef PIPE_AUX_ST
#define PIPE_AUX_ST GEMM_ST_AUX
#endif
__device__ __forceinline__ i32x4_t c_rsrc(const GemmArgs& a) {
    const size_t bytes = (size_t)((a.M + 15) & ~15) * a.ldc * 2;  // (blocked C: rows padded to 16)
    return buf_rsrc(a.C, (unsigned)(bytes < 0xFFFFFFFFu ? bytes : 0xFFFFFFFFu));
}
__device__ __forceinline__ void c_store(unsigned char* Cb, const i32x4_t& rs, size_t off, const uint4& v) {
    if constexpr (PIPE_AUX_ST == 0) *(uint4*)(Cb + off) = v;
    else st16_pol<PIPE_AUX_ST>(rs, off, v);
}

template <typename T, int BM, int BN, int WM, int WN, int NS, int EPI, int SM = 0, int PIMPL = 0>
__global__ __launch_bounds__(64 * WM* WN, WM* WN >= 4 ? 2 : 4) void gemm_pipe_kernel(GemmArgs a) {
    typedef typename T::vec8 vec8;
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    static_assert(TN % 64 == 0 && TM % 16 == 0, "wave tile");
    constexpr int A_BYTES = BM * 128, W_BYTES = BN * 128;
    // staging rounds; a last partial round (e.g. BM = 160) is issued by whole waves only, which
    // makes per-wave load counts differ -> allowed only with NS = 2 (waits are vmcnt(0) there)
    constexpr int LA = (A_BYTES + NT * 16 - 1) / (NT * 16), LW = (W_BYTES + NT * 16 - 1) / (NT * 16);
    constexpr bool PARTIAL = LA * NT * 16 != A_BYTES || LW * NT * 16 != W_BYTES;
    static_assert(!PARTIAL || NS == 2, "partial staging rounds need NS == 2");
    static_assert(A_BYTES % 1024 == 0 && W_BYTES % 1024 == 0, "whole-wave staging pieces");
    constexpr int LPT = LA + LW;  // glds per thread per tile (upper bound when PARTIAL)
    constexpr int STAGE = A_BYTES + W_BYTES;
    // epilogue operands staged in LDS at kernel start (their global loads overlap the prologue):
    // per-column bias / b' and s (LNF), per-row mu / rstd (LNF) — the epilogue then issues no
    // dependent global loads
    constexpr bool LNF = EPI == EPI_LNF || EPI == EPI_LNF_GELU;
    constexpr bool COLV = EPI == EPI_STORE || EPI == EPI_GELU || LNF || EPI == EPI_RES_STATS;
    constexpr int EXTRA = COLV ? 2 * BN * 4 + (LNF ? BM * 8 : 0) : 0;
    static_assert(BN <= NT && BM <= NT, "one column / row of epilogue operands per thread");
    __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STAGE + EXTRA];
    float* const colv = (float*)(smem + NS * STAGE);  // [BN] bias or b', [BN] s
    float* const rowv = colv + 2 * BN;                // [BM] (mu, rstd)

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int nN = a.N / BN;
    int mt, nt;
    if (!tile_of_block(blockIdx.x, (a.M + BM - 1) / BM, nN, a.xcd_n, mt, nt)) return;
    const int m0 = mt * BM, n0 = nt * BN;

    const unsigned char* Ab = (const unsigned char*)a.A;
    const unsigned char* Wb = (const unsigned char*)a.W;
    const size_t ldb = (size_t)a.K * 2;
    const int mlast = a.M - 1;
    // per-thread source row offsets (constant over k)
    size_t asrc[LA], wsrc[LW];
    int acol[LA];  // PIMPL: the piece's (swizzled) 16-B chunk inside the 64-wide k-tile
#pragma unroll
    for (int r = 0; r < LA; ++r) {
        const int p = r * NT * 16 + tid * 16;
        const int row = p >> 7, c = ((p >> 4) & 7) ^ (row & 7);
        if constexpr (PIMPL > 0) {
            constexpr int PP = (PIMPL + 7) / 8 * 8;
            const int m = min(m0 + row, mlast), R = a.patch_R, Rw = a.patch_Rw, G = R / PIMPL;
            const int b = m / a.patch_g2, pp = m - b * a.patch_g2, py = pp / G, px = pp - py * G;
            asrc[r] = ((size_t)b * 3 * R * Rw + (size_t)py * PIMPL * Rw + px * PP) * 2;
            acol[r] = c;
        } else {
            asrc[r] = (size_t)min(m0 + row, mlast) * ldb + c * 16;
            acol[r] = 0;
        }
    }
#pragma unroll
    for (int r = 0; r < LW; ++r) {
        const int p = r * NT * 16 + tid * 16;
        const int row = p >> 7, c = ((p >> 4) & 7) ^ (row & 7);
        wsrc[r] = (size_t)(n0 + row) * ldb + c * 16;
    }
    // split-K slice (EPI_F32 only, launch_pipe): k-tiles [kz * nk, kz * nk + nk) of the row
    const int kz = a.ksplit > 1 ? (int)blockIdx.y : 0;
    const size_t kbase = a.ksplit > 1 ? (size_t)kz * (a.K / a.ksplit) * 2 : 0;
    // Staging by buffer loads over the tile's own rows (resource base = first row of the tile):
    // the 32-bit per-lane offsets stay constant over k and the k offset is an SGPR, so a k-step
    // issues no address arithmetic (global_load_lds needed a 64-bit add per piece; measured
    // B/32 bs 256 83.3k -> 83.9k img/s, c_proj 0.739 -> 0.723 ms per forward).
    // Implicit-GEMM patches with P | 64 and 64 | P^2 (P = 16, 32): a 64-deep k-tile is 64 / P
    // whole pixel rows of one channel, so a piece's pixel offset = a per-lane part (row inside
    // the k-tile, 8-pixel chunk) + a wave-uniform part of kt (channel, first row): the same
    // buffer-load form, resource based at the tile's first image. P = 14 keeps per-lane
    // patch_koff addresses (its channels are 224 k long: k-tiles straddle channels).
    constexpr bool PSEP = PIMPL > 0 && 64 % PIMPL == 0 && (PIMPL * PIMPL) % 64 == 0;
    constexpr bool BUFL = PIMPL == 0 || PSEP;
    i32x4_t rsA{}, rsW{};
    unsigned boa[BUFL ? LA : 1], bow[BUFL ? LW : 1];
    if constexpr (BUFL) {
        const size_t wbytes = (size_t)(a.N - n0) * ldb;
        rsW = buf_rsrc(Wb + (size_t)n0 * ldb, (unsigned)min(wbytes, (size_t)0xFFFFFFFFu));
        if (a.blk_w) {  // blocked W (blk16_off over the packed rows): the blk_a form below
#pragma unroll
            for (int r = 0; r < LW; ++r) {
                const int p = r * NT * 16 + tid * 16;
                bow[r] = (unsigned)((size_t)(p >> 11) * 16 * ldb + (p & 2047));
            }
        } else {
#pragma unroll
            for (int r = 0; r < LW; ++r) bow[r] = (unsigned)(wsrc[r] - (size_t)n0 * ldb);
        }
        if constexpr (PSEP) {
            constexpr int CPR = PIMPL / 8;  // 16-B chunks per pixel row of a patch
            const size_t img = (size_t)3 * a.patch_R * a.patch_Rw * 2;  // bytes per image
            const int b0 = min(m0, mlast) / a.patch_g2, nimg = a.M / a.patch_g2;
            rsA = buf_rsrc(Ab + b0 * img, (unsigned)min((size_t)(nimg - b0) * img, (size_t)0xFFFFFFFFu));
#pragma unroll
            for (int r = 0; r < LA; ++r)
                boa[r] = (unsigned)(asrc[r] - b0 * img + 2 * ((acol[r] / CPR) * a.patch_Rw + 8 * (acol[r] % CPR)));
        } else if (a.blk_a) {
            // 16-row blocked A (blk16_off): the stage's LDS image is chunk-major per 16-row block,
            // i.e. each block's 2 KB k-tile run copied verbatim (row blocks past the last one
            // clamped; rows past M inside it are padding and only feed unstored output rows)
            const int mpad = (a.M + 15) & ~15, lastb = (mpad - m0) / 16 - 1;
            const size_t abytes = (size_t)(mpad - m0) * ldb;
            rsA = buf_rsrc(Ab + (size_t)m0 * ldb, (unsigned)min(abytes, (size_t)0xFFFFFFFFu));
#pragma unroll
            for (int r = 0; r < LA; ++r) {
                const int p = r * NT * 16 + tid * 16;
                boa[r] = (unsigned)((size_t)min(p >> 11, lastb) * 16 * ldb + (p & 2047));
            }
        } else {
            const size_t abytes = (size_t)(a.M - m0) * ldb;
            rsA = buf_rsrc(Ab + (size_t)m0 * ldb, (unsigned)min(abytes, (size_t)0xFFFFFFFFu));
#pragma unroll
            for (int r = 0; r < LA; ++r) boa[r] = (unsigned)(asrc[r] - (size_t)m0 * ldb);
        }
    }
    auto stage = [&](int buf, int kt) {
        unsigned char* sA = smem + buf * STAGE;
        unsigned char* sW = sA + A_BYTES;
        const size_t kofs = kbase + (size_t)kt * 128;
        if constexpr (BUFL) {
            int aofs = a.blk_a ? kt * 2048 : (int)kofs;  // (blk_a / blk_w: no split-K, launch_pipe)
            const int wofs = a.blk_w ? kt * 2048 : (int)kofs;
            if constexpr (PSEP) {  // channel kt / KPC, first pixel row (kt % KPC) * (64 / P)
                constexpr int KPC = PIMPL * PIMPL / 64;
                aofs = ((kt / KPC) * a.patch_R + (kt % KPC) * (64 / PIMPL)) * a.patch_Rw * 2;
            }
#pragma unroll
            for (int r = 0; r < LA; ++r)
                if (r * NT * 16 + wave * 1024 < A_BYTES) blds16(rsA, boa[r], aofs, sA + r * NT * 16 + wave * 1024);
#pragma unroll
            for (int r = 0; r < LW; ++r)
                if (r * NT * 16 + wave * 1024 < W_BYTES) blds16(rsW, bow[r], wofs, sW + r * NT * 16 + wave * 1024);
            return;
        }
#pragma unroll
        for (int r = 0; r < LA; ++r)
            if (r * NT * 16 + wave * 1024 < A_BYTES)  // wave-uniform
                glds16(Ab + asrc[r] + 2 * (size_t)patch_koff<PIMPL>(kt * 64 + 8 * acol[r], a.patch_R, a.patch_Rw),
                       sA + r * NT * 16 + wave * 1024);
#pragma unroll
        for (int r = 0; r < LW; ++r)
            if (r * NT * 16 + wave * 1024 < W_BYTES)
                glds16(Wb + wsrc[r] + kofs, sW + r * NT * 16 + wave * 1024);
    };

    const int lrow = lane & 15, lsw = lane & 7, lg = lane >> 4;
    // A fragment of row lrow, k-chunk (s << 2) | lg: swizzled row-major image, or (blk_a) the
    // chunk-major image of the 16-row blocks (chunk * 256 + row * 16, conflict-free unswizzled)
    const bool ablk = a.blk_a != 0, wblk = BUFL && a.blk_w != 0;
    const int aoff = ablk ? wm * TM * 128 + lrow * 16 : (wm * TM + lrow) * 128;
    const int woff = A_BYTES + (wblk ? wn * TN * 128 + lrow * 16 : (wn * TN + lrow) * 128);
    auto load_frags = [&](int buf, int s, vec8 (&af)[FM], vec8 (&wf)[FN]) {
        const unsigned char* base = smem + buf * STAGE;
        const int c = (((s << 2) | lg) ^ lsw) << 4;
        const int ca = ablk ? ((s << 2) | lg) << 8 : c;
        const int cw = wblk ? ((s << 2) | lg) << 8 : c;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) af[fm] = *(const vec8*)(base + aoff + fm * 2048 + ca);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) wf[fn] = *(const vec8*)(base + woff + fn * 2048 + cw);
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Ring protocol: tile t lives in stage t % NS. Prologue issues tiles 0..NS-2; the stage of
    // tile t-1 is refilled with tile t-1+NS right after the barrier that follows every wave's
    // last ds_read of tile t-1 (lgkmcnt(0) before that barrier).
    const int nk = (a.ksplit > 1 ? a.K / a.ksplit : a.K) >> 6;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) stage(s, s);
    // epilogue operands: issued behind the prologue's loads (their first use waits for vmcnt(0),
    // which with NS = 2 is the prologue's own wait)
    float cb = 0.f, cs = 0.f;
    float2 stv[LNF ? 8 : 1];  // np <= 8: width <= 1024 (clipvit_create)
    if constexpr (COLV) {
        if (tid < BN) {
            if (a.bias) cb = a.bias[n0 + tid];
            if constexpr (LNF) cs = a.lnf_s[n0 + tid];
        }
    }
    if constexpr (LNF) {
        const float2* st = a.st_in + (size_t)min(m0 + tid, mlast) * a.np;
#pragma unroll
        for (int p = 0; p < 8; ++p) stv[p] = st[min(p, a.np - 1)];  // unconditional loads (no per-load branch)
    }
    wait_tile<LPT, NS>(min(NS - 2, nk - 1));
    if constexpr (COLV) {
        if (tid < BN) {
            colv[tid] = cb;
            colv[BN + tid] = cs;
        }
    }
    if constexpr (LNF) {
        if (tid < BM) {
            float s = 0.f;
#pragma unroll
            for (int p = 0; p < 8; ++p) s += p < a.np ? stv[p].x : 0.f;
            const float mu = s / (float)a.np;
            float m2 = 0.f;
#pragma unroll
            for (int p = 0; p < 8; ++p)
                if (p < a.np) {
                    const float d = stv[p].x - mu;
                    m2 += stv[p].y + 128.f * d * d;
                }
            rowv[2 * tid] = mu;
            rowv[2 * tid + 1] = rsqrtf(m2 / (128.f * (float)a.np) + 1e-5f);
        }
    }
    __builtin_amdgcn_s_barrier();
    if (NS - 1 < nk) stage(NS - 1, NS - 1);

    constexpr int NFR = FM + FN;        // ds_read_b128 per substep
    constexpr int NMF = FM * FN;        // MFMAs per substep
    // interleave the NFR reads of the next substep one-per-MFMA among this substep's MFMAs
    auto interleave = [&]() {
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NMF - NFR, 0);
    };
    static_assert(NMF >= NFR, "need at least one MFMA per fragment read");
    auto mfmas = [&](const vec8 (&af)[FM], const vec8 (&wf)[FN]) {
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) acc[fn][fm] = T::mfma16(wf[fn], af[fm], acc[fn][fm]);
    };

    vec8 a0[FM], w0[FN], a1[FM], w1[FN];
    load_frags(0, 0, a0, w0);
    for (int kt = 0; kt < nk - 1; ++kt) {   // steady state: branch-free around the LDS reads
        const int cur = kt % NS;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): a0/w0 (read one MFMA block ago) landed
        load_frags(cur, 1, a1, w1);
        mfmas(a0, w0);
        interleave();
        __builtin_amdgcn_s_waitcnt(0xC07F);                  // a1/w1 landed: stage kt fully read
        wait_tile<LPT, NS>(min(NS - 2, nk - 2 - kt));       // tile kt+1 landed (own loads)
        __builtin_amdgcn_s_barrier();                        // ... and everyone else's
        if (kt + NS < nk) stage(cur, kt + NS);               // refill the stage just freed
        load_frags((kt + 1) % NS, 0, a0, w0);
        mfmas(a1, w1);
        interleave();
    }
    // EPI_RES_STATS: the residual rows this lane updates are loaded during the last tile's MFMAs
    // (prefetched where the registers allow: FM <= 5, i.e. the 160-row tiles of the N = 768 roles)
    constexpr bool PREX = EPI == EPI_RES_STATS && FM <= 5;
    float4 xpre[PREX ? FM : 1][4];
    {   // last tile
        __builtin_amdgcn_s_waitcnt(0xC07F);
        load_frags((nk - 1) % NS, 1, a1, w1);
        if constexpr (PREX) {
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) {
                const int m = min(m0 + wm * TM + fm * 16 + lrow, mlast);
                const size_t idx = (size_t)m * a.ldc + n0 + wn * TN + 16 * lg;
                if (a.x24_plane) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) xpre[fm][i] = x24_load((const unsigned char*)a.C, a.x24_plane, idx + 4 * i);
                } else {
                    const float4* xr = (const float4*)((const float*)a.C + idx);
#pragma unroll
                    for (int i = 0; i < 4; ++i) xpre[fm][i] = xr[i];
                }
            }
        }
        mfmas(a0, w0);
        interleave();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        mfmas(a1, w1);
    }

    // ---- epilogue (same contract as gemm_nt_kernel) ----
    const int g = lg;
    constexpr bool GELU = EPI == EPI_GELU || EPI == EPI_F32GELU || EPI == EPI_LNF_GELU;
    if constexpr (SM == 3 && (EPI == EPI_STORE || EPI == EPI_GELU || LNF)) {
        // Row-contiguous stores staged through LDS: the accumulator layout gives each lane 32 B
        // of one row, so direct stores cover 16 rows x 4 scattered 16-B pieces per
        // wave-instruction; here the tile is first written to LDS (row-major, 16-B chunk
        // c ^ (row & 7): conflict-free ds_write_b128), then every wave-instruction stores whole
        // rows (64 lanes x 16 B contiguous).
        constexpr int ROWB = BN * 2, CPR = ROWB / 16;
        static_assert(BM * ROWB <= NS * STAGE, "epilogue tile must fit in the LDS ring");
        __builtin_amdgcn_s_barrier();  // every wave is done reading the ring
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
            const int r = wm * TM + fm * 16 + lrow;
            float mu = 0.f, rstd = 1.f;
            if constexpr (LNF) {
                mu = rowv[2 * r];
                rstd = rowv[2 * r + 1];
            }
#pragma unroll
            for (int q = 0; q < FN / 4; ++q) {
                const int nl = wn * TN + q * 64 + 16 * g;
                float v[16];
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) v[4 * f + rr] = acc[4 * q + f][fm][rr];
                if constexpr (LNF) lnf_apply(v, colv + BN + nl, colv + nl, mu, rstd);
                else colv_add(v, colv + nl);
                if constexpr (GELU) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) v[i] = quick_gelu(v[i]);
                }
                const int c0 = nl >> 3;  // 16-B chunk of the row
                unsigned char* rowp = smem + r * ROWB;
                *(uint4*)(rowp + (((c0) ^ (r & 7)) << 4)) =
                    make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7]));
                *(uint4*)(rowp + (((c0 + 1) ^ (r & 7)) << 4)) =
                    make_uint4(pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]), pack2<T>(v[12], v[13]), pack2<T>(v[14], v[15]));
            }
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_s_barrier();
        unsigned char* Cb = (unsigned char*)a.C;
        const i32x4_t rs_c = c_rsrc(a);
        if (a.blk_c) {  // blocked C: a quarter-wave stores one chunk of 16 rows (256 B contiguous)
#pragma unroll 4
            for (int i = tid; i < BM * CPR; i += NT) {
                const int r = ((i >> 4) / CPR) * 16 + (i & 15), c = (i >> 4) % CPR;
                const int m = m0 + r;
                const uint4 val = *(const uint4*)(smem + r * ROWB + ((c ^ (r & 7)) << 4));
                if (m < a.M) c_store(Cb, rs_c, blk16_off(m, n0 + 8 * c, a.ldc), val);
            }
            return;
        }
#pragma unroll 4
        for (int i = tid; i < BM * CPR; i += NT) {
            const int r = i / CPR, c = i % CPR;
            const int m = m0 + r;
            const uint4 val = *(const uint4*)(smem + r * ROWB + ((c ^ (r & 7)) << 4));
            if (m < a.M) c_store(Cb, rs_c, ((size_t)m * a.ldc + n0) * 2 + c * 16, val);
        }
        return;
    }
    unsigned char* const Cb = (unsigned char*)a.C + (EPI == EPI_F32 ? (size_t)kz * a.M * a.ldc * 4 : 0);
    if constexpr (EPI == EPI_RES_STATS) {
        res_stats_epilogue<T, FM, FN, TM, TN, WN, PREX>(a, acc, xpre, colv + wn * TN + 16 * lg, smem, m0, n0, wm, wn,
                                                        lane);
        return;
    }
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
        const int m = m0 + wm * TM + fm * 16 + lrow;
        if (m >= a.M) continue;
        float mu = 0.f, rstd = 1.f;
        if constexpr (LNF) {
            const int r = m - m0;
            mu = rowv[2 * r];
            rstd = rowv[2 * r + 1];
        }
#pragma unroll
        for (int q = 0; q < FN / 4; ++q) {
            const int n = n0 + wn * TN + q * 64 + 16 * g;
            float v[16];
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[4 * f + r] = acc[4 * q + f][fm][r];
            if constexpr (LNF) {
                lnf_apply(v, colv + BN + (n - n0), colv + (n - n0), mu, rstd);
            } else if constexpr (COLV) {
                colv_add(v, colv + (n - n0));
            } else if constexpr (EPI != EPI_PATCH) {
                if (a.bias) {
                    const float4* b4 = (const float4*)(a.bias + n);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float4 bb = b4[i];
                        v[4 * i] += bb.x; v[4 * i + 1] += bb.y; v[4 * i + 2] += bb.z; v[4 * i + 3] += bb.w;
                    }
                }
            }
            if constexpr (GELU) {
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = quick_gelu(v[i]);
            }
            if constexpr (EPI == EPI_STORE || EPI == EPI_GELU || LNF) {
                // blocked C: n % 16 == 0, so n + 8 is the next chunk of the same 64-block (+256 B)
                const size_t off = a.blk_c ? blk16_off(m, n, a.ldc) : ((size_t)m * a.ldc + n) * 2;
                const size_t off2 = a.blk_c ? off + 256 : off + 16;
                const i32x4_t rs_c = c_rsrc(a);
                c_store(Cb, rs_c, off, make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]),
                                                  pack2<T>(v[6], v[7])));
                c_store(Cb, rs_c, off2, make_uint4(pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]),
                                                   pack2<T>(v[12], v[13]), pack2<T>(v[14], v[15])));
            } else if constexpr (EPI == EPI_RESID) {
                const float4* src = (const float4*)((float*)a.C + (size_t)m * a.ldc + n);
                const size_t off = ((size_t)m * a.ldc + n) * 4;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float4 o = src[i];
                    o.x += v[4 * i]; o.y += v[4 * i + 1]; o.z += v[4 * i + 2]; o.w += v[4 * i + 3];
                    *(float4*)(Cb + off + 16 * i) = o;
                }
            } else {
                size_t row = (size_t)m;
                if constexpr (EPI == EPI_PATCH)
                    row = (size_t)(m / a.patch_g2) * a.patch_ntok + 1 + (m % a.patch_g2);
                const size_t off = (row * a.ldc + n) * 4;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    *(float4*)(Cb + off + 16 * i) = (make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]));
            }
        }
    }
}

template <typename T, int BM, int BN, int WM, int WN, int NS, int SM = 0>
static int launch_pipe(hipStream_t s, int epi, const GemmArgs& a) {
    const int nwg = grid_for((a.M + BM - 1) / BM, a.N / BN, a.xcd_n);
    if (a.ksplit > 1 && (epi != EPI_F32 || a.K % (64 * a.ksplit) != 0)) return -1;
    dim3 grid(nwg, a.ksplit > 1 ? a.ksplit : 1), block(64 * WM * WN);
#define PIPE(E) gemm_pipe_kernel<T, BM, BN, WM, WN, NS, E, SM><<<grid, block, 0, s>>>(a)
    switch (epi) {
        case EPI_STORE: PIPE(EPI_STORE); return 0;
        case EPI_GELU: PIPE(EPI_GELU); return 0;
        case EPI_RESID: PIPE(EPI_RESID); return 0;
        case EPI_LNF: PIPE(EPI_LNF); return 0;
        case EPI_LNF_GELU: PIPE(EPI_LNF_GELU); return 0;
        case EPI_RES_STATS:
            if constexpr (BN / WN == 64 && WN % 2 == 0) {
                PIPE(EPI_RES_STATS);
                return 0;
            }
            return -1;  // statistics groups need 64-wide waves in pairs
        case EPI_F32: PIPE(EPI_F32); return 0;
        case EPI_F32GELU: PIPE(EPI_F32GELU); return 0;
        case EPI_PATCH:
            if constexpr (SM == 0) {
                PIPE(EPI_PATCH);
                return 0;
            }
            return -1;
    }
#undef PIPE
    return -1;
}

// Implicit-GEMM patch embedding on 160x128 tiles (4 waves, two workgroups per CU: the v22 tile
// of the im2col path); a.A = 16-bit pixels [B, 3, R, Rw], a.K = padded patch length,
// a.patch_R = R, a.patch_Rw = pixel row length (R, or G * 16 for P = 14).
template <typename T>
static int launch_patch_t(hipStream_t s, int P, const GemmArgs& a) {
    if (a.N % 128) return -1;
    const int nwg = grid_for((a.M + 159) / 160, a.N / 128, a.xcd_n);
    switch (P) {
        case 14: gemm_pipe_kernel<T, 160, 128, 2, 2, 2, EPI_PATCH, 0, 14><<<nwg, 256, 0, s>>>(a); return 0;
        case 16: gemm_pipe_kernel<T, 160, 128, 2, 2, 2, EPI_PATCH, 0, 16><<<nwg, 256, 0, s>>>(a); return 0;
        case 32: gemm_pipe_kernel<T, 160, 128, 2, 2, 2, EPI_PATCH, 0, 32><<<nwg, 256, 0, s>>>(a); return 0;
    }
    return -1;
}
int launch_patch_gemm(hipStream_t s, int dtype, int P, const GemmArgs& a) {
    return dtype == 2 ? launch_patch_t<F16>(s, P, a) : launch_patch_t<BF16>(s, P, a);
}

// 16-bit -> fp32 copy (test entry for the 16-bit-output kernels)
template <typename T>
__global__ void widen16_kernel(const u16* src, float* dst, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = T::to_f32(src[i]);
}
void launch_widen16(hipStream_t s, int dtype, const void* src, float* dst, size_t n) {
    const unsigned g = (unsigned)((n + 255) / 256);
    if (dtype == 2) widen16_kernel<F16><<<g, 256, 0, s>>>((const u16*)src, dst, n);
    else widen16_kernel<BF16><<<g, 256, 0, s>>>((const u16*)src, dst, n);
}

template <typename T, int BM, int BN, int WM, int WN>
static int launch_tile(hipStream_t s, int epi, const GemmArgs& a) {
    const int nwg = (a.N / BN) * ((a.M + BM - 1) / BM);
    dim3 grid(nwg), block(64 * WM * WN);
    switch (epi) {
        case EPI_STORE: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_STORE><<<grid, block, 0, s>>>(a); return 0;
        case EPI_GELU: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_GELU><<<grid, block, 0, s>>>(a); return 0;
        case EPI_RESID: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_RESID><<<grid, block, 0, s>>>(a); return 0;
        case EPI_PATCH: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_PATCH><<<grid, block, 0, s>>>(a); return 0;
        case EPI_F32: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_F32><<<grid, block, 0, s>>>(a); return 0;
        case EPI_F32GELU: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_F32GELU><<<grid, block, 0, s>>>(a); return 0;
    }
    return -1;  // the LayerNorm-fold / statistics epilogues live in the pipelined kernel only
}

// Auto tile choice: the largest tile whose grid still covers the 256 CUs reasonably.
static int pick_variant(const GemmArgs& a) {
    const long t256 = (long)(a.N % 256 == 0 ? a.N / 256 : 0) * ((a.M + 255) / 256);
    const long t256x128 = (long)(a.N / 128) * ((a.M + 255) / 256);
    if (t256 >= 400) return 3;
    if (a.N % 128 == 0 && t256x128 >= 400) return 2;
    return 1;
}

template <typename T>
static int launch_t(hipStream_t s, int epi, const GemmArgs& a, int variant) {
    if (variant == 0) variant = pick_variant(a);
    switch (variant) {
        // ---- single-buffer-per-k-step tiles: shape fallback (pick_variant) ----
        case 1:
            if (a.N % 128) return -1;
            return launch_tile<T, 128, 128, 2, 2>(s, epi, a);
        case 2:
            if (a.N % 128) return -1;
            return launch_tile<T, 256, 128, 4, 2>(s, epi, a);
        case 3:
            if (a.N % 256) return -1;
            return launch_tile<T, 256, 256, 2, 4>(s, epi, a);
        // ---- pipelined ring tiles (the production roles, clipvit.hip gemm()) ----
        case 8:   // 256x256, 8 waves: main launch of the c_fc round split
            if (a.N % 256) return -1;
            return launch_pipe<T, 256, 256, 2, 4, 2>(s, epi, a);
        case 22:  // 160x128, 4 waves, two workgroups per CU: patch embedding
            if (a.N % 128) return -1;
            return launch_pipe<T, 160, 128, 2, 2, 2>(s, epi, a);
        // ---- LDS-staged row-contiguous 16-bit epilogue (SM = 3) ----
        case 81:  // 128x128: tail launch of the c_fc round split
            if (a.N % 128) return -1;
            return launch_pipe<T, 128, 128, 4, 2, 2, 3>(s, epi, a);
        case 82:  // 160x128, two workgroups per CU: out_proj / c_proj
            if (a.N % 128) return -1;
            return launch_pipe<T, 160, 128, 2, 2, 2, 3>(s, epi, a);
        case 98:  // 240x256, 12 waves (3 x 4, 80 x 64 per wave): QKV (486 tiles = 1.9 rounds at bs 256)
            if (a.N % 256) return -1;
            return launch_pipe<T, 240, 256, 3, 4, 2, 3>(s, epi, a);
        // ---- 64x64 tiles, 4-stage ring: the class-token tail's M = B GEMMs ----
        case 90:
            if (a.N % 64) return -1;
            return launch_pipe<T, 64, 64, 2, 1, 4>(s, epi, a);
    }
    return -1;
}

int launch_gemm(hipStream_t s, int dtype, int epi, const GemmArgs& a, int variant) {
    if (a.K % 64 != 0 || a.M <= 0) return -1;
    if (a.blk_a || a.blk_c) {  // blocked u / h: pipelined 8..98 and persistent 62 / 72 / 74 / 75 / 77 / 79 only
        if (variant < 8 || a.ksplit > 1) return -1;
        if (a.blk_c && (a.ldc % 64 || (epi != EPI_STORE && epi != EPI_GELU && epi != EPI_LNF && epi != EPI_LNF_GELU)))
            return -1;
    }
    // blocked W: the pipelined tiles and the persistent tiles (62 / 72 / 74 / 75 / 77 / 79)
    if (a.blk_w && (variant < 8 || a.ksplit > 1)) return -1;
    if (variant == 62 || variant == 72 || variant == 74 || variant == 75 || variant == 77 || variant == 79)
        return launch_gemm_pp(s, dtype, epi, a, variant);
    // split-K runs on the pipelined tiles only (launch_pipe checks the epilogue and K)
    if (a.ksplit > 1 && variant < 8) return -1;
    if (dtype == 2) return launch_t<F16>(s, epi, a, variant);
    return launch_t<BF16>(s, epi, a, variant);
}

}  // namespace clipvit
