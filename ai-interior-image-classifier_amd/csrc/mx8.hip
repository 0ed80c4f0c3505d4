// MX-fp8 path of the encoder's dense contractions (BASELINE.json config 5: fp8 weights, 16-bit
// activations between kernels, fp32 residual / LayerNorm / softmax).
//
// Format (OCP MX): e4m3 elements, one E8M0 power-of-two scale per 32 consecutive K-elements of
// a row. Weights are quantized once at load time (launch_pack_weight_mx8, same 64-row
// permutation as the 16-bit packer); GEMM A-operands are quantized by their producers —
// LayerNorm (ln_1 / ln_2 -> qkv / c_fc), the c_fc epilogue (QuickGELU -> c_proj) and
// launch_quant_mx8 (attention output -> out_proj). The GEMM runs on
// v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate, block scales applied in hardware).
//
// GEMM kernel = gemm_pipe_kernel's structure (glds 128-B rows, 2-stage LDS ring, swapped
// operands so a lane owns 16 contiguous output features) at BK = 128 fp8 per k-step:
//  * operand lane map (measured on MI355X, tools/probes/mx_probe.hip): lane l, g = l >> 4,
//    holds row l & 15 at k = 16 g + j (bytes j < 16) and k = 64 + 16 g + j - 16 (bytes
//    j >= 16), i.e. 16-B chunks g and g + 4 of the 128-B row; the E8M0 scale operand of lane
//    r + 16 b applies to row r, k-block b (= k / 32) -> a lane passes the scale of block g;
//  * LDS rows are 128 B; 16-B chunk c of row r lives at c ^ (r & 7): chunks g and g + 4 are
//    the 16-bit kernel's two k-substeps (c = 4 s + g), conflict-free for ds_read_b128;
//  * per k-step each stage also receives the 4 scale bytes (one dword) of every A and W row
//    by 4-byte glds; a lane reads its byte with ds_read_u8.
#include <algorithm>
#include <type_traits>
#include "common.h"
#include "gemm_p32mx.h"

namespace clipvit {

typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int mx_sw(int r) { return r & 7; }

// ---------------------------------------------------------------------------------------
// 16-bit (or fp32) [rows][K] -> MX-fp8; one thread per 32-element block.
template <int IN>
__global__ void quant_mx8_kernel(const void* __restrict__ src, unsigned char* __restrict__ q,
                                 unsigned char* __restrict__ sq, long nblk) {
    const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    float v[32];
    if constexpr (IN == 0) {
        const float4* p = (const float4*)src + b * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 t = p[i];
            v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
        }
    } else {
        const uint4* p = (const uint4*)src + b * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 t = p[i];
            const unsigned w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u16 lo = (u16)(w[j] & 0xffff), hi = (u16)(w[j] >> 16);
                v[8 * i + 2 * j] = IN == 1 ? BF16::to_f32(lo) : F16::to_f32(lo);
                v[8 * i + 2 * j + 1] = IN == 1 ? BF16::to_f32(hi) : F16::to_f32(hi);
            }
        }
    }
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) a = fmaxf(a, fabsf(v[i]));
    const int e = mx_exp(a);
    const float inv = mx_inv(e);
    unsigned o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = pk4_e4m3(v[4 * i] * inv, v[4 * i + 1] * inv, v[4 * i + 2] * inv, v[4 * i + 3] * inv);
    uint4* d = (uint4*)q + b * 2;
    d[0] = make_uint4(o[0], o[1], o[2], o[3]);
    d[1] = make_uint4(o[4], o[5], o[6], o[7]);
    sq[b] = (unsigned char)(e + 127);
}

void launch_quant_mx8(hipStream_t s, int in_dtype, const void* src, unsigned char* q,
                      unsigned char* sq, int rows, int K) {
    const long nblk = (long)rows * (K / 32);
    const unsigned g = (unsigned)((nblk + 255) / 256);
    if (in_dtype == 0) quant_mx8_kernel<0><<<g, 256, 0, s>>>(src, q, sq, nblk);
    else if (in_dtype == 2) quant_mx8_kernel<2><<<g, 256, 0, s>>>(src, q, sq, nblk);
    else quant_mx8_kernel<1><<<g, 256, 0, s>>>(src, q, sq, nblk);
}

// Benchmark operands: uniform [-1, 1) values as e4m3 with unit block scales.
__global__ void fill_random_mx8_kernel(unsigned char* q, unsigned char* sq, size_t n, unsigned seed) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n / 4) return;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        unsigned x = (unsigned)(4 * i + j) * 2654435761u ^ (seed * 0x9E3779B9u);
        x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
        v[j] = (float)(x >> 8) * (2.0f / 16777216.0f) - 1.0f;
    }
    ((unsigned*)q)[i] = pk4_e4m3(v[0], v[1], v[2], v[3]);
    if ((4 * i) % 32 == 0) sq[4 * i / 32] = 127;
}

void launch_fill_random_mx8(hipStream_t s, unsigned char* q, unsigned char* sq, size_t n, unsigned seed) {
    fill_random_mx8_kernel<<<(unsigned)((n / 4 + 255) / 256), 256, 0, s>>>(q, sq, n, seed);
}

// fp32 [N][K] Linear weight -> MX-fp8 [N][Kp] + scales [N][Kp/32], rows permuted inside each
// 64-row group exactly as pack_weight_kernel (norm.hip); columns >= K are zero.
__global__ void pack_weight_mx8_kernel(const float* __restrict__ src, unsigned char* __restrict__ q,
                                       unsigned char* __restrict__ sq, int N, int K, int Kp) {
    const long b = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int nb = Kp / 32;
    if (b >= (long)N * nb) return;
    const int p = (int)(b / nb), kb = (int)(b % nb);
    const int grp = p & ~63, pi = p & 63, f = pi >> 4, i = pi & 15;
    const int n = grp + 16 * (i >> 2) + 4 * f + (i & 3);
    float v[32];
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const int k = kb * 32 + j;
        v[j] = k < K ? src[(size_t)n * K + k] : 0.f;
        a = fmaxf(a, fabsf(v[j]));
    }
    const int e = mx_exp(a);
    const float inv = mx_inv(e);
    unsigned o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = pk4_e4m3(v[4 * j] * inv, v[4 * j + 1] * inv, v[4 * j + 2] * inv, v[4 * j + 3] * inv);
    uint4* d = (uint4*)(q + (size_t)p * Kp + kb * 32);
    d[0] = make_uint4(o[0], o[1], o[2], o[3]);
    d[1] = make_uint4(o[4], o[5], o[6], o[7]);
    sq[(size_t)p * nb + kb] = (unsigned char)(e + 127);
}

void launch_pack_weight_mx8(hipStream_t s, const float* src, unsigned char* q, unsigned char* sq,
                            int N, int K, int Kp) {
    const long nblk = (long)N * (Kp / 32);
    pack_weight_mx8_kernel<<<(unsigned)((nblk + 255) / 256), 256, 0, s>>>(src, q, sq, N, K, Kp);
}

// ---------------------------------------------------------------------------------------
// C[M, N] = dequant(A8)[M, K] @ dequant(W8)[N, K]^T (+ bias), fused epilogue.
template <typename TO, int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(64 * WM* WN, 2) void gemm_mx8_kernel(GemmArgs a) {
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    static_assert(TN % 64 == 0 && TM % 16 == 0, "wave tile");
    constexpr int A_BYTES = BM * 128, W_BYTES = BN * 128;
    constexpr int LA = (A_BYTES + NT * 16 - 1) / (NT * 16), LW = (W_BYTES + NT * 16 - 1) / (NT * 16);
    static_assert(A_BYTES % 1024 == 0 && W_BYTES % 1024 == 0, "whole-wave staging pieces");
    constexpr int SC_ROWS = BM + BN;                      // one scale dword per row per k-step
    // every wave issues SCW 4-byte scale glds per k-step (branch-free; SCW = 2 when the tile has
    // more rows than threads, e.g. 160x128 on 4 waves); lanes past the last scale row fill a pad
    constexpr int SCW = (SC_ROWS + NT - 1) / NT;
    constexpr int STAGE = A_BYTES + W_BYTES + SCW * NT * 4;
    static_assert(LA * NT * 16 == A_BYTES && LW * NT * 16 == W_BYTES, "whole staging rounds");
    // one LDS object per ring stage: with the stage index a compile-time constant at every
    // use, alias analysis separates the stage being refilled by LDS-DMA from the one being
    // read, and the compiler does not guard the fragment ds_reads with vmcnt(0)
    __shared__ __attribute__((aligned(16))) unsigned char smem0[STAGE];
    __shared__ __attribute__((aligned(16))) unsigned char smem1[STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int nN = a.N / BN;
    int mt, nt;
    if (!tile_of_block(blockIdx.x, (a.M + BM - 1) / BM, nN, a.xcd_n, mt, nt)) return;
    const int m0 = mt * BM, n0 = nt * BN;

    const unsigned char* Ab = (const unsigned char*)a.A;
    const unsigned char* Wb = (const unsigned char*)a.W;
    const size_t ldb = (size_t)a.K;          // fp8 row stride in bytes
    const size_t lds_ = (size_t)(a.K / 32);  // scale row stride
    const int mlast = a.M - 1;
    unsigned asrc[LA], wsrc[LW];  // byte offsets (operands < 4 GiB)
#pragma unroll
    for (int r = 0; r < LA; ++r) {
        const int p = r * NT * 16 + tid * 16;
        const int row = p >> 7, c = ((p >> 4) & 7) ^ mx_sw(row & 15);
        asrc[r] = (unsigned)((size_t)min(m0 + row, mlast) * ldb + c * 16);
    }
#pragma unroll
    for (int r = 0; r < LW; ++r) {
        const int p = r * NT * 16 + tid * 16;
        const int row = p >> 7, c = ((p >> 4) & 7) ^ mx_sw(row & 15);
        wsrc[r] = (unsigned)((size_t)(n0 + row) * ldb + c * 16);
    }
    // scale rows: thread t loads the dwords of rows t (and t + NT when SCW = 2; A rows first,
    // then W rows; rows >= SC_ROWS: pad)
    static_assert(SCW <= 2, "at most two scale dwords per thread");
    auto scale_row = [&](int r) -> const unsigned char* {
        return r < BM ? a.sA + (size_t)min(m0 + r, mlast) * lds_
             : r < SC_ROWS ? a.sW + (size_t)(n0 + r - BM) * lds_
                           : a.sW + (size_t)n0 * lds_;
    };
    const unsigned char* ssrc = scale_row(tid);
    const unsigned char* ssrc2 = scale_row(tid + NT);

    // operand staging by buffer loads: constant 32-bit per-lane offsets, k offset in an SGPR
    // (same scheme as gemm_pipe_kernel)
    const i32x4_t rsA = buf_rsrc(Ab, (unsigned)min((size_t)a.M * ldb, (size_t)0xFFFFFFFFu));
    const i32x4_t rsW = buf_rsrc(Wb, (unsigned)min((size_t)a.N * ldb, (size_t)0xFFFFFFFFu));
    auto stage = [&](auto B, int kt) {
        unsigned char* sA = decltype(B)::value ? smem1 : smem0;
        unsigned char* sW = sA + A_BYTES;
        unsigned char* sS = sW + W_BYTES;
        const int kofs = kt * 128;
#pragma unroll
        for (int r = 0; r < LA; ++r) blds16(rsA, asrc[r], kofs, sA + r * NT * 16 + wave * 1024);
#pragma unroll
        for (int r = 0; r < LW; ++r) blds16(rsW, wsrc[r], kofs, sW + r * NT * 16 + wave * 1024);
        __builtin_amdgcn_global_load_lds((const GLB_AS void*)(ssrc + kt * 4),
                                         (LDS_AS void*)(sS + wave * 256), 4, 0, 0);
        if constexpr (SCW == 2)
            __builtin_amdgcn_global_load_lds((const GLB_AS void*)(ssrc2 + kt * 4),
                                             (LDS_AS void*)(sS + NT * 4 + wave * 256), 4, 0, 0);
    };

    const int lrow = lane & 15, lg = lane >> 4;
    // fragment addresses: rows of a lane's fragments differ by multiples of 16, so the
    // swizzle depends on lrow only and every fragment is base + compile-time offset
    const int fsw = mx_sw(lrow);
    const int c0 = (lg ^ fsw) << 4, c1 = ((lg + 4) ^ fsw) << 4;
    const int fa = (wm * TM + lrow) * 128;
    const int fw = A_BYTES + (wn * TN + lrow) * 128;
    const int fsa = A_BYTES + W_BYTES + (wm * TM + lrow) * 4 + lg;
    const int fsw_ = A_BYTES + W_BYTES + (BM + wn * TN + lrow) * 4 + lg;
    auto frag = [&](const unsigned char* p) -> i32x8 {
        const uint4 lo = *(const uint4*)(p + c0);
        const uint4 hi = *(const uint4*)(p + c1);
        return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    };
    constexpr int FH = FN / 2;  // W fragments per half k-step
    static_assert(FN % 2 == 0, "two W halves");
    auto load_a = [&](auto B, i32x8 (&af)[FM], int (&as)[FM]) {
        const unsigned char* sb = decltype(B)::value ? smem1 : smem0;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
            af[fm] = frag(sb + fa + fm * 2048);
            as[fm] = sb[fsa + fm * 64];
        }
    };
    auto load_w = [&](auto B, int half, i32x8 (&wf)[FH], int (&ws)[FH]) {
        const unsigned char* sb = decltype(B)::value ? smem1 : smem0;
#pragma unroll
        for (int j = 0; j < FH; ++j) {
            const int fn = half * FH + j;
            wf[j] = frag(sb + fw + fn * 2048);
            ws[j] = sb[fsw_ + fn * 64];
        }
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mfmas = [&](int half, const i32x8 (&af)[FM], const int (&as)[FM], const i32x8 (&wf)[FH],
                     const int (&ws)[FH]) {
#pragma unroll
        for (int j = 0; j < FH; ++j)
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
                acc[half * FH + j][fm] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                    wf[j], af[fm], acc[half * FH + j][fm], 0, 0, 0, ws[j], 0, as[fm]);
    };
    // interleave n reads (3 instructions per fragment) one-per-MFMA into a block of FH*FM MFMAs
    auto interleave = [&](auto NRD) {
        constexpr int nrd = decltype(NRD)::value;
#pragma unroll
        for (int i = 0; i < FH * FM; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (i < nrd) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if constexpr (nrd > FH * FM) __builtin_amdgcn_sched_group_barrier(0x100, nrd - FH * FM, 0);
    };

    // K-step kt (stage kt & 1) runs as two MFMA blocks over the two W halves, exactly like the
    // 16-bit pipe kernel's two k-substeps: block 0 runs while the second W half is read;
    // then, after the barrier that hands over stage kt+1 (and frees stage kt for k-step kt+2),
    // block 1 runs while the next step's A fragments and first W half are read.
    // Registers: A fragments x2 (current, next), W halves x2, accumulators.
    const int nk = a.K >> 7;
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    stage(P0{}, 0);
    vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (nk > 1) stage(P1{}, 1);
    i32x8 a0[FM], a1[FM], wl[FH], wh[FH];
    int sa0[FM], sa1[FM], swl[FH], swh[FH];
    load_a(P0{}, a0, sa0);
    load_w(P0{}, 0, wl, swl);

    // k-step with a successor (kt + 1 < nk)
    auto kstep = [&](int kt, auto P, i32x8 (&ac)[FM], int (&sac)[FM], i32x8 (&an)[FM], int (&san)[FM]) {
        constexpr int cur = decltype(P)::value;
        using PN = std::integral_constant<int, cur ^ 1>;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // A fragments + first W half of stage kt landed
        load_w(P, 1, wh, swh);
        mfmas(0, ac, sac, wl, swl);
        interleave(std::integral_constant<int, 3 * FH>{});
        __builtin_amdgcn_s_waitcnt(0xC07F);  // stage kt fully read
        vm_wait<0>();                        // stage kt+1 landed (own loads)
        __builtin_amdgcn_s_barrier();        // ... everyone's; nobody reads stage kt any more
        // branch-free: past the end the freed stage is refilled with a real (unused) k-step,
        // which keeps the loop body one basic block (no MFMA sinking past the barriers)
        stage(P, min(kt + 2, nk - 1));
        load_a(PN{}, an, san);
        load_w(PN{}, 0, wl, swl);
        mfmas(1, ac, sac, wh, swh);
        interleave(std::integral_constant<int, 3 * (FM + FH)>{});
    };
    auto klast = [&](auto P, i32x8 (&ac)[FM], int (&sac)[FM]) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        load_w(P, 1, wh, swh);
        mfmas(0, ac, sac, wl, swl);
        interleave(std::integral_constant<int, 3 * FH>{});
        __builtin_amdgcn_s_waitcnt(0xC07F);
        mfmas(1, ac, sac, wh, swh);
    };
    int kt = 0;
    for (; kt + 2 < nk; kt += 2) {  // pairs of k-steps that both have a successor
        kstep(kt, P0{}, a0, sa0, a1, sa1);
        kstep(kt + 1, P1{}, a1, sa1, a0, sa0);
    }
    if (kt + 2 == nk) {
        kstep(kt, P0{}, a0, sa0, a1, sa1);
        klast(P1{}, a1, sa1);
    } else {
        klast(P0{}, a0, sa0);
    }

    // ---- epilogue: lane (lrow, g) owns token m, 16 contiguous features n .. n+15 ----
    const int g = lg;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
        const int m = m0 + wm * TM + fm * 16 + lrow;
#pragma unroll
        for (int q = 0; q < FN / 4; ++q) {
            const int n = n0 + wn * TN + q * 64 + 16 * g;
            float v[16];
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[4 * f + r] = acc[4 * q + f][fm][r];
            if (a.bias) {
                const float4* b4 = (const float4*)(a.bias + n);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float4 bb = b4[i];
                    v[4 * i] += bb.x; v[4 * i + 1] += bb.y; v[4 * i + 2] += bb.z; v[4 * i + 3] += bb.w;
                }
            }
            if constexpr (EPI == EPI_GELU_Q8 || EPI == EPI_F32GELU) {
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = quick_gelu(v[i]);
            }
            if constexpr (EPI == EPI_GELU_Q8 || EPI == EPI_Q8) {
                // MX block = 32 features = this lane's 16 + those of lane ^ 16 (same token)
                float am = 0.f;
#pragma unroll
                for (int i = 0; i < 16; ++i) am = fmaxf(am, fabsf(v[i]));
                am = fmaxf(am, __shfl_xor(am, 16, 64));
                if (m >= a.M) continue;
                const int e = mx_exp(am);
                const float inv = mx_inv(e);
                // blocked C (blk_c, blk8_off): the quarter-wave's 16 rows x 16 B are 256 contiguous bytes
                cstore16<MX_AUX_ST>(a.C, a.blk_c ? blk8_off(m, n, a.ldc) : (size_t)m * a.ldc + n,
                    make_uint4(pk4_e4m3(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv),
                               pk4_e4m3(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv),
                               pk4_e4m3(v[8] * inv, v[9] * inv, v[10] * inv, v[11] * inv),
                               pk4_e4m3(v[12] * inv, v[13] * inv, v[14] * inv, v[15] * inv)));
                if ((g & 1) == 0)
                    a.sC[a.sc_rows ? ((size_t)(n >> 7) * a.sc_rows + m) * 4 + ((n >> 5) & 3)
                                   : (size_t)m * (a.ldc / 32) + (n >> 5)] = (unsigned char)(e + 127);
                continue;
            }
            if (m >= a.M) continue;
            if constexpr (EPI == EPI_STORE) {
                uint4* dst = (uint4*)((u16*)a.C + (size_t)m * a.ldc + n);
                dst[0] = make_uint4(pack2<TO>(v[0], v[1]), pack2<TO>(v[2], v[3]), pack2<TO>(v[4], v[5]),
                                    pack2<TO>(v[6], v[7]));
                dst[1] = make_uint4(pack2<TO>(v[8], v[9]), pack2<TO>(v[10], v[11]),
                                    pack2<TO>(v[12], v[13]), pack2<TO>(v[14], v[15]));
            } else if constexpr (EPI == EPI_RESID) {
                float4* dst = (float4*)((float*)a.C + (size_t)m * a.ldc + n);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float4 o = dst[i];
                    o.x += v[4 * i]; o.y += v[4 * i + 1]; o.z += v[4 * i + 2]; o.w += v[4 * i + 3];
                    dst[i] = o;
                }
            } else {  // EPI_F32 / EPI_F32GELU
                float4* dst = (float4*)((float*)a.C + (size_t)m * a.ldc + n);
#pragma unroll
                for (int i = 0; i < 4; ++i) dst[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
            }
        }
    }
}

template <typename TO, int BM, int BN, int WM, int WN>
static int launch_mx8_tile(hipStream_t s, int epi, const GemmArgs& a) {
    if (a.N % BN) return -1;
    const int nwg = grid_for((a.M + BM - 1) / BM, a.N / BN, a.xcd_n);
    dim3 grid(nwg), block(64 * WM * WN);
    switch (epi) {
        case EPI_STORE: gemm_mx8_kernel<TO, BM, BN, WM, WN, EPI_STORE><<<grid, block, 0, s>>>(a); break;
        case EPI_RESID: gemm_mx8_kernel<TO, BM, BN, WM, WN, EPI_RESID><<<grid, block, 0, s>>>(a); break;
        case EPI_GELU_Q8: gemm_mx8_kernel<TO, BM, BN, WM, WN, EPI_GELU_Q8><<<grid, block, 0, s>>>(a); break;
        case EPI_Q8: gemm_mx8_kernel<TO, BM, BN, WM, WN, EPI_Q8><<<grid, block, 0, s>>>(a); break;
        case EPI_F32: gemm_mx8_kernel<TO, BM, BN, WM, WN, EPI_F32><<<grid, block, 0, s>>>(a); break;
        case EPI_F32GELU: gemm_mx8_kernel<TO, BM, BN, WM, WN, EPI_F32GELU><<<grid, block, 0, s>>>(a); break;
        default: return -1;
    }
    return 0;
}

// ---------------------------------------------------------------------------------------
// Ping-pong MX-fp8 tile (variant 3, persistent): gemm_ppp_kernel's
// schedule (gemm_pp.hip, profiles/design_r05.md §5.8) at BK = 128 fp8. A k-tile row is 128 B in both
// formats, so the LDS layout, the staging pieces and the phase/slot plan are the 16-bit
// kernel's; per phase a wave runs 8 scaled 16x16x128 MFMAs (2x the cycles of the 16-bit form,
// so the same matrix-pipe time per phase as the 16 bf16 MFMAs it replaces). Each stage also
// carries the 4 scale bytes of every A and W row (2 KB): the wave that issues part 0 of its
// group's operand stages the scale dwords of 64 rows with one 4-byte buffer_load ... lds, so
// part 0 is 3 VMEM ops and the counted waits are 3 (group 0) / 5 (group 1). Scale rows are
// read with their fragments (A: q0, q2; W: q0, q1) and refilled with part 0 (group 1 at q2,
// group 0 at q3), after the last read of each.
template <typename TO, int EPI, bool BLKA = false, bool BLKC = false>
__global__ __launch_bounds__(512, 1) void gemm_mx8_pp_kernel(GemmArgs a, int ntiles) {
    constexpr int BM = 256, BN = 256;
    constexpr int A_BYTES = BM * 128, OPS = (BM + BN) * 128, STAGE = OPS + (BM + BN) * 4;  // 66 KB
    constexpr int NBIAS = 4096;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE + NBIAS * 4];  // 148 KB
    float* const colv = (float*)(smem + 2 * STAGE);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int nM = (a.M + BM - 1) / BM, nN = a.N / BN;
    const int G = gridDim.x;
    const size_t ldb = (size_t)a.K, lds_ = (size_t)(a.K / 32);
    const int nk = a.K >> 7;  // even, >= 2 (launcher)

    auto tile = [&](int i, int& m0, int& n0) {
        const int L = blockIdx.x + i * G;
        if (L >= ntiles) return false;
        int mt, nt;
        tile_of_block(L, nM, nN, a.xcd_n, mt, nt);
        m0 = mt * BM;
        n0 = nt * BN;
        return true;
    };
    const unsigned char* src = (const unsigned char*)(grp == 0 ? a.A : a.W);
    const unsigned char* ssrc = grp == 0 ? a.sA : a.sW;
    const int rows = grp == 0 ? a.M : a.N;
    // blocked A (blk_a, blk8_off; rows padded to 16): piece pc of the A stage is half pc & 1 of
    // 16-row block pc >> 1, whose 128-deep k-tile is one contiguous 2 KB run (chunk-major image)
    // (BLKA: a compile-time choice. As a runtime flag the compiler kept both voff sets alive and
    // spilled them in the QuickGELU + quantize instantiation; the reloads, VMEM ops under the
    // in-order vmcnt, then waited for every staging load in flight)
    const bool ablk = BLKA && grp == 0;
    const int orows = ablk ? (a.M + 15) & ~15 : rows;
    auto rsrc_of = [&](int m0, int n0) {
        const int r0 = grp == 0 ? m0 : n0;
        const size_t bytes = (size_t)(orows - r0) * ldb;
        return buf_rsrc(src + (size_t)r0 * ldb, (unsigned)(bytes < 0xFFFFFFFFu ? bytes : 0xFFFFFFFFu));
    };
    // scale dwords: one resource over the whole scale array (rows past M / N read 0), the
    // tile's row offset in the per-lane offset (VGPRs: the SGPR budget is spent). Blocked A
    // scales (sc_rows): [K / 128][sc_rows] dwords, so the k-tile offset is kk * sc_rows * 4 and
    // a wave's 64 rows are one 256-B run (row-major: 64 dwords K / 32 bytes apart)
    const bool sblk = BLKA && grp == 0 && a.sc_rows;
    const i32x4_t ssr = buf_rsrc(ssrc, (unsigned)(sblk ? (size_t)a.sc_rows * (a.K / 128) * 4 : (size_t)rows * lds_));
    const int sk_stride = sblk ? a.sc_rows * 4 : 4;  // bytes per k-tile
    auto svoff_of = [&](int m0, int n0) {
        const int r = (grp == 0 ? m0 : n0) + wc * 64 + lane;
        return (unsigned)(sblk ? (size_t)r * 4 : (size_t)r * lds_);
    };
    const int lr = lane >> 3, chunk = (lane & 7) ^ lr;
    // 32-bit offset arithmetic (a tile's operand rows span < 4 GB): 64-bit products here were kept
    // as register pairs and spilled in the QuickGELU + quantize instantiation
    const unsigned ldb32 = (unsigned)ldb;
    unsigned voff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const unsigned pc = 8 * (i >> 1) + 2 * wc + (i & 1);
        voff[i] = ablk ? (pc >> 1) * 16u * ldb32 + (pc & 1) * 1024u + (unsigned)lane * 16u
                       : (pc * 8u + (unsigned)lr) * ldb32 + (unsigned)chunk * 16u;
    }
    const int kshift = ablk ? 11 : 7;  // bytes per k-tile along a row (block): 2048 / 128
    const unsigned obase = (grp == 0 ? 0 : A_BYTES) + 2 * wc * 1024;  // + (8 part + i) KB
    const unsigned sbase = OPS + grp * BM * 4 + wc * 256;

    int m0, n0, mn = 0, nn = 0;
    tile(0, m0, n0);  // the launcher sizes the grid <= ntiles
    bool has_next = tile(1, mn, nn);
    i32x4_t rs_c = rsrc_of(m0, n0), rs_n = has_next ? rsrc_of(mn, nn) : rs_c;
    unsigned sv_c = svoff_of(m0, n0), sv_n = has_next ? svoff_of(mn, nn) : sv_c;
    // k-tile j of the current tile's frame (j >= nk: k-tile j - nk of the next tile)
    // S: the stage k-tile j lands in (= j & 1, nk even), a compile-time constant at every call
    // so that the LDS destinations are immediates (m0), not SGPRs
    auto issue = [&](int part, int j, auto S) {
        i32x4_t r = rs_c;
        unsigned sv = sv_c;
        int kk = j;
        if (j >= nk) {
            if (!has_next) return;
            r = rs_n;
            sv = sv_n;
            kk = j - nk;
        }
        // the wave's LDS offsets, opaque per call: otherwise the compiler hoists all 18 m0
        // values of the loop into SGPRs and spills (the destinations stay smem-based pointers,
        // which keeps the fragment ds_reads free of compiler-inserted vmcnt(0))
        unsigned ob = obase, sb = sbase;
        asm volatile("" : "+s"(ob), "+s"(sb));
        constexpr unsigned so = decltype(S)::value * STAGE;
#pragma unroll
        for (int i = 0; i < 2; ++i) blds16(r, voff[2 * part + i], kk << kshift, smem + ob + so + (8 * part + i) * 1024);
        if (part == 0) raw_buffer_load_lds(ssr, (LDS_AS void*)(smem + sb + so), 4, (int)sv, kk * sk_stride, 0, 0);
    };

    f32x4 acc[4][8];
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
#pragma unroll
    for (int p = 0; p < 4; ++p) issue(p, 0, S0{});
    if (grp == 0) {
        issue(0, 1, S1{});
    } else {
        issue(0, 1, S1{});
        issue(1, 1, S1{});
    }
    for (int i = tid; i < a.N; i += 512) colv[i] = a.bias ? a.bias[i] : 0.f;
    if (grp == 0) vm_wait<3>(); else vm_wait<5>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger

    // lane-derived LDS read addresses: re-derived per tile from an opaque lane id (asm, so
    // neither it nor they are loop-invariant). Held across the whole persistent loop they
    // get spilled, and their reload at a tile's first read waits for every staging load.
    auto lane_id = [] {
        int l;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
        return l;
    };
    int aoff, woff, asoff, wsoff, c0, c1, ca0, ca1, sshift;
    auto lane_addrs = [&] {
        const int l = lane_id();
        const int lrow = l & 15, lsw = l & 7, lg = l >> 4;
        // A: swizzled row-major image, or (blk_a) chunk-major 16-row blocks
        aoff = BLKA ? grp * 128 * 128 + lrow * 16 : (grp * 128 + lrow) * 128;
        ca0 = BLKA ? lg << 8 : ((0 | lg) ^ lsw) << 4;
        ca1 = BLKA ? (4 | lg) << 8 : ((4 | lg) ^ lsw) << 4;
        woff = A_BYTES + (wc * 64 + lrow) * 128;
        asoff = OPS + (grp * 128 + lrow) * 4;
        wsoff = OPS + BM * 4 + (wc * 64 + lrow) * 4;
        c0 = ((0 | lg) ^ lsw) << 4;
        c1 = ((4 | lg) ^ lsw) << 4;
        sshift = 8 * lg;  // the lane's scale byte (k-block lg) within the row's dword
    };
    i32x8 af[4], wf[4];
    int as[4], ws[4];
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    // fragment and scale reads through non-char types: with char / unsigned-int typed LDS reads
    // the compiler cannot tell them apart from the pending LDS-DMA writes and puts vmcnt(0) in
    // front of every read phase (the 16-bit kernel's bf16x8 reads do not have that problem)
    auto frag = [&](const unsigned char* p, int o0, int o1) -> i32x8 {
        const i32x4_t lo = __builtin_bit_cast(i32x4_t, *(const bf16x8*)(p + o0));
        const i32x4_t hi = __builtin_bit_cast(i32x4_t, *(const bf16x8*)(p + o1));
        return i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    };
    auto scale = [&](const unsigned char* p) -> int {
        return (int)((__builtin_bit_cast(unsigned, *(const float*)p) >> sshift) & 0xffu);
    };
    auto mfmas = [&](auto FN0, auto FM0, auto Zc) {
        constexpr int fn0 = decltype(FN0)::value, fm0 = decltype(FM0)::value;
#pragma unroll
        for (int fn = fn0; fn < fn0 + 2; ++fn)
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
                acc[fn][fm + fm0] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                    wf[fn], af[fm], decltype(Zc)::value ? zero : acc[fn][fm + fm0], 0, 0, 0, ws[fn], 0, as[fm]);
        // pin the block to its phase: the MFMA intrinsics are pure, and without a use here IR
        // sinking moves them past the barriers (into the next phases' read segments)
#pragma unroll
        for (int fn = fn0; fn < fn0 + 2; ++fn)
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) asm volatile("" : "+v"(acc[fn][fm + fm0]));
    };
    using I0 = std::integral_constant<int, 0>;
    using I2 = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, 4>;

    auto ktile = [&](const int kt, auto Pc, auto Zc) {
        constexpr int P = decltype(Pc)::value;  // kt & 1
        using PS = std::integral_constant<int, P>;
        using NS = std::integral_constant<int, P ^ 1>;
        const unsigned char* st = smem + P * STAGE;
        const bool more = kt + 2 < nk || has_next;
        // q0: W features 0-31, A rows 0-63 of the wave's half
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            wf[f] = frag(st + woff + f * 2048, c0, c1);
            ws[f] = scale(st + wsoff + f * 64);
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            af[f] = frag(st + aoff + f * 2048, ca0, ca1);
            as[f] = scale(st + asoff + f * 64);
        }
        if (grp == 0) issue(1, kt + 1, NS{}); else issue(2, kt + 1, NS{});
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        mfmas(I0{}, I0{}, Zc);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        // q1: W features 32-63 (last W read of this stage)
#pragma unroll
        for (int f = 2; f < 4; ++f) {
            wf[f] = frag(st + woff + f * 2048, c0, c1);
            ws[f] = scale(st + wsoff + f * 64);
        }
        if (grp == 0) issue(2, kt + 1, NS{}); else issue(3, kt + 1, NS{});
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        mfmas(I2{}, I0{}, Zc);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        // q2: A rows 64-127 (last A read of this stage)
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            af[f] = frag(st + aoff + (f + 4) * 2048, ca0, ca1);
            as[f] = scale(st + asoff + (f + 4) * 64);
        }
        if (grp == 0) issue(3, kt + 1, NS{}); else issue(0, kt + 2, PS{});
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        mfmas(I2{}, I4{}, Zc);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        // q3: no reads
        if (grp == 0) {
            issue(0, kt + 2, PS{});
        } else {
            issue(1, kt + 2, PS{});
            if (more) vm_wait<5>(); else vm_wait<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
        mfmas(I0{}, I4{}, Zc);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (grp == 0) {
            if (more) vm_wait<3>(); else vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();
    };

    for (int i = 1;; ++i) {
        lane_addrs();
        ktile(0, S0{}, std::true_type{});
        ktile(1, S1{}, std::false_type{});
        for (int kt = 2; kt < nk; kt += 2) {
            ktile(kt, S0{}, std::false_type{});
            ktile(kt + 1, S1{}, std::false_type{});
        }
        // epilogue (as gemm_ppp_kernel: bias from LDS by inline-asm reads, no vmcnt drain). The
        // lane coordinates are re-derived from an opaque, recomputed lane id: loop-invariant
        // epilogue addresses hoisted out of the persistent loop get spilled (the k-loop holds
        // 255 VGPRs), and a scratch reload here would wait for the next tile's staging loads
        const int ln = lane_id();
        const int er = ln & 15, eg = ln >> 4;
        const int n = n0 + wc * 64 + 16 * eg;
        // blocked u8 (BLKC): offsets of the lane's row at fm = 0; fm steps 16 rows = one block
        // row (cbs bytes) and 16 scale dwords
        unsigned cb0 = 0, cbs = 0, sb0 = 0;
        if constexpr (BLKC) {
            const int mr = m0 + grp * 128 + er;
            cb0 = (unsigned)blk8_off(mr, n, a.ldc);
            cbs = (unsigned)(a.ldc >> 7) << 11;
            sb0 = ((unsigned)(n >> 7) * (unsigned)a.sc_rows + (unsigned)mr) * 4u + (unsigned)((n >> 5) & 3);
        }
        f32x4 bv[4];
        {
            const unsigned ba = (unsigned)(size_t)(LDS_AS const float*)(colv + n);
            asm volatile("ds_read_b128 %0, %1" : "=v"(bv[0]) : "v"(ba) : "memory");
            asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(bv[1]) : "v"(ba) : "memory");
            asm volatile("ds_read_b128 %0, %1 offset:32" : "=v"(bv[2]) : "v"(ba) : "memory");
            asm volatile("ds_read_b128 %0, %1 offset:48" : "=v"(bv[3]) : "v"(ba) : "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int fm = 0; fm < 8; ++fm) {
            const int m = m0 + grp * 128 + fm * 16 + er;
            float v[16];
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) v[4 * f + rr] = acc[f][fm][rr] + bv[f][rr];
            if constexpr (EPI == EPI_GELU_Q8) {
#pragma unroll
                for (int q = 0; q < 16; ++q) v[q] = quick_gelu(v[q]);
                // MX block = 32 features = this lane's 16 + those of lane ^ 16 (same token):
                // ds_swizzle bitmask mode, xor 0x10 within 32-lane groups (no address VGPR)
                float am = 0.f;
#pragma unroll
                for (int q = 0; q < 16; ++q) am = fmaxf(am, fabsf(v[q]));
                am = fmaxf(am, __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(am), 0x401F)));
                const int e = mx_exp(am);
                const float inv = mx_inv(e);
                if (m < a.M) {
                    // blocked C (BLKC = blk_c, compile-time: the runtime choice spilled the
                    // accumulators): the quarter-wave's 16 rows x 16 B are 256 contiguous bytes;
                    // its scales [K / 128][sc_rows] dwords. 32-bit offsets (< 4 GB), fm-strided
                    unsigned co, so;
                    if constexpr (BLKC) {
                        co = cb0 + (unsigned)fm * cbs;
                        so = sb0 + (unsigned)fm * 64u;
                    } else {
                        co = (unsigned)m * (unsigned)a.ldc + (unsigned)n;
                        so = (unsigned)m * (unsigned)(a.ldc / 32) + (unsigned)(n >> 5);
                    }
                    cstore16<MX_AUX_ST>(a.C, co,
                        make_uint4(pk4_e4m3(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv),
                                   pk4_e4m3(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv),
                                   pk4_e4m3(v[8] * inv, v[9] * inv, v[10] * inv, v[11] * inv),
                                   pk4_e4m3(v[12] * inv, v[13] * inv, v[14] * inv, v[15] * inv)));
                    if ((eg & 1) == 0) a.sC[so] = (unsigned char)(e + 127);
                }
            } else if (m < a.M) {  // EPI_STORE
                const size_t off = ((size_t)m * a.ldc + n) * 2;
                cstore16<MX_AUX_ST16>(a.C, off, make_uint4(pack2<TO>(v[0], v[1]), pack2<TO>(v[2], v[3]),
                                                         pack2<TO>(v[4], v[5]), pack2<TO>(v[6], v[7])));
                cstore16<MX_AUX_ST16>(a.C, off + 16, make_uint4(pack2<TO>(v[8], v[9]), pack2<TO>(v[10], v[11]),
                                                              pack2<TO>(v[12], v[13]), pack2<TO>(v[14], v[15])));
            }
        }
        if (!has_next) break;
        m0 = mn;
        n0 = nn;
        rs_c = rs_n;
        sv_c = sv_n;
        has_next = tile(i + 1, mn, nn);
        if (has_next) {
            rs_n = rsrc_of(mn, nn);
            sv_n = svoff_of(mn, nn);
        }
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
}

template <typename TO>
static int launch_mx8_pp(hipStream_t s, int epi, const GemmArgs& a, bool persistent) {
    if (a.N % 256 || a.K % 256 || a.N > 4096 || xcd_split_n(a.N / 256, a.xcd_n)) return -1;
    const int ncu = a.ncu > 0 ? a.ncu : 256;
    const int ntiles = ((a.M + 255) / 256) * (a.N / 256);
    const int grid = persistent && ntiles > ncu ? ncu : ntiles;
    if (epi == EPI_STORE && a.blk_a) { gemm_mx8_pp_kernel<TO, EPI_STORE, true><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_STORE) { gemm_mx8_pp_kernel<TO, EPI_STORE><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_GELU_Q8 && !a.blk_a) {
        if (a.blk_c != (a.sc_rows != 0)) return -1;  // blocked u8 goes with its blocked scales
        if (a.blk_c) gemm_mx8_pp_kernel<TO, EPI_GELU_Q8, false, true><<<grid, 512, 0, s>>>(a, ntiles);
        else gemm_mx8_pp_kernel<TO, EPI_GELU_Q8><<<grid, 512, 0, s>>>(a, ntiles);
        return 0;
    }
    return -1;
}

// Variant 4: gemm_p32mx.h (the 32x32x64 scaled MFMA on the 4-stage 64-deep-k-step ring), balanced
// persistent grid (the fewest workgroups with the same tiles per workgroup). Row-major A.
template <typename TO>
static int launch_mx8_p32(hipStream_t s, int epi, const GemmArgs& a) {
    if (a.N % 256 || a.N > 4096 || a.K % 256 || a.K < 512 || a.blk_a || xcd_split_n(a.N / 256, a.xcd_n)) return -1;
    if ((size_t)(a.M + 15) * a.ldc * 4 >= 0xFFFFFFC0u) return -1;  // 32-bit epilogue offsets
    const int ncu = a.ncu > 0 ? a.ncu : 256;
    const int ntiles = ((a.M + 255) / 256) * (a.N / 256);
    const int per = (ntiles + ncu - 1) / ncu;
    const int grid = (ntiles + per - 1) / per;
    if (epi == EPI_STORE && !a.blk_c) { gemm_mx8_p32_kernel<TO, EPI_STORE, false><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_F32 && !a.blk_c) { gemm_mx8_p32_kernel<TO, EPI_F32, false><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_F32GELU && !a.blk_c) { gemm_mx8_p32_kernel<TO, EPI_F32GELU, false><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_GELU_Q8) {
        if (a.blk_c != (a.sc_rows != 0)) return -1;  // blocked u8 goes with its blocked scales
        if (a.blk_c) gemm_mx8_p32_kernel<TO, EPI_GELU_Q8, true><<<grid, 512, 0, s>>>(a, ntiles);
        else gemm_mx8_p32_kernel<TO, EPI_GELU_Q8, false><<<grid, 512, 0, s>>>(a, ntiles);
        return 0;
    }
    return -1;
}

// variant: 0 auto, 1 128x256 (2x4 waves), 2 128x128 (2x2 waves), 3 ping-pong 256x256
// persistent, 5 160x128 (2x2 waves; two per CU,
// 480 tiles = one round at M = 12,800, N = 768)
template <typename TO>
static int launch_mx8_t(hipStream_t s, int epi, const GemmArgs& a, int variant) {
    if (variant == 0) variant = a.N % 256 == 0 ? 1 : 2;
    switch (variant) {
        case 1: return launch_mx8_tile<TO, 128, 256, 2, 4>(s, epi, a);
        case 2: return launch_mx8_tile<TO, 128, 128, 2, 2>(s, epi, a);
        case 3: return launch_mx8_pp<TO>(s, epi, a, true);
        case 4: return launch_mx8_p32<TO>(s, epi, a);
        case 5: return launch_mx8_tile<TO, 160, 128, 2, 2>(s, epi, a);
    }
    return -1;
}

int launch_gemm_mx8(hipStream_t s, int out16, int epi, const GemmArgs& a, int variant) {
    if (a.K % 128 != 0 || a.M <= 0 || !a.sA || !a.sW) return -1;
    // blocked u8: read by the persistent ping-pong only; written by it or (c_fc tail launch of
    // the whole-round row split) by the 128 x 128 / 160 x 128 tiles' QuickGELU + quantize epilogue
    if (a.blk_a && variant != 3) return -1;
    if (a.blk_c && variant != 3 && variant != 4 && variant != 2 && variant != 5) return -1;
    if (a.blk_c && (epi != EPI_GELU_Q8 || a.ldc % 128)) return -1;
    if ((epi == EPI_GELU_Q8 || epi == EPI_Q8) && (!a.sC || a.ldc % 32)) return -1;
    if (out16 == 2) return launch_mx8_t<F16>(s, epi, a, variant);
    return launch_mx8_t<BF16>(s, epi, a, variant);
}

}  // namespace clipvit
