// Ping-pong MFMA GEMM: 256x256 tiles, 8 waves in two wave groups staggered by one barrier,
// persistent (one workgroup per CU; variants 62 / 63). Diagnostic forms of this kernel (stamps,
// ablations) live in tools/probes/gemm_probe.hip, not here.
//
//   C[M, N] = A[M, K] @ W[N, K]^T + bias (16-bit C; QuickGELU for c_fc)
//
// Same operand conventions as gemm.hip (K-major A and packed W, swapped MFMA operands so a lane
// owns one token and 16 contiguous features, LDS rows of 128 B with 16-B chunk c of row r at
// c ^ (r & 7)), different schedule (profiles/design_r05.md §5.8):
//
//  * waves 0-3 (group 0) and 4-7 (group 1) each own 128 token rows x 64 features per wave
//    (wave w: rows 128 (w >> 2) .., features 64 (w & 3) ..); each SIMD hosts one wave of each
//    group. Every 64-deep k-tile is four phases (one 64x32 quadrant of the wave's tile each,
//    16 MFMAs): [LDS fragment reads + LDS-DMA issue] barrier [MFMAs] barrier. Group 1 runs one
//    barrier behind group 0, so on every SIMD one wave's MFMAs cover the other wave's reads,
//    DMA issue and barrier wait, and the matrix pipe is never idle at a barrier;
//  * operand staging by buffer_load ... lds into two 64 KB stages; the loads of k-tile j are
//    spread over the six phases in which their LDS rows are free (group 0 stages A, group 1
//    stages W, two 1-KB pieces per wave per phase) and waited for by counted vmcnt — never 0
//    in the loop — so they stay in flight across barriers;
//  * schedule (slot = barrier interval; group g's phase P reads in slot 2P + g and runs its
//    MFMAs in 2P + g + 1): W of a stage is last read in phase q1, A rows of group g in q2, so
//    k-tile j + 2 may refill stage j & 1 from slot 8j + 5 (W) / 8j + 6 (A rows of group 0) /
//    8j + 7 (group 1); every issuing wave waits for its pieces before the barrier that opens
//    the first read of that k-tile (the end of slot 8j + 7 for k-tile j + 1).
#include <type_traits>

#include "common.h"
#include "gemm_p32.h"

namespace clipvit {

// ---------------------------------------------------------------------------------------
// Persistent form (variant 62): one workgroup per CU walks the tiles blockIdx.x, blockIdx.x + G,
// ... (G = grid size; logical ids through the same bijective XCD remap, so every XCD group
// keeps a contiguous range of the row-major tile order each round). The k-tile stream runs on
// across tile boundaries: the last phases of a tile already stage the next tile's first two
// k-tiles, so a tile's prologue load never stalls the CU, and the finished tile's epilogue
// (bias, QuickGELU, 16-bit stores straight from the accumulators) runs in the first read
// segment of the next tile while the other wave group's MFMAs go on. The bias vector of the
// whole GEMM (N <= 8192) is parked in the 32 KB of LDS beside the two stages.

template <typename T, int EPI, bool NT = false, bool BLKA = false, bool BLKW = false>
__global__ __launch_bounds__(512, 1) void gemm_ppp_kernel(GemmArgs a, int ntiles) {
    typedef typename T::vec8 vec8;
    constexpr int BM = 256, BN = 256;
    constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
    constexpr int NBIAS = 8192;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE + NBIAS * 4];  // 160 KB
    float* const colv = (float*)(smem + 2 * STAGE);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    const int nM = (a.M + BM - 1) / BM, nN = a.N / BN;
    const int G = gridDim.x;
    const size_t ldb = (size_t)a.K * 2;
    const int nk = a.K >> 6;  // even, >= 2

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
    // blocked A (blk_a, blk16_off; rows padded to 16): piece pc of the A stage is half pc & 1 of
    // 16-row block pc >> 1, whose k-tile run is contiguous — the LDS image is chunk-major
    // (BLKA compile-time: a runtime flag keeps both per-lane offset sets alive)
    // blocked W (BLKW, GemmArgs.blk_w): the same form for the weight group's pieces
    const bool ablk = BLKA && grp == 0;
    const bool oblk = ablk || (BLKW && grp == 1);  // this group's staged operand is blocked
    const int rows = grp == 0 ? (BLKA ? (a.M + 15) & ~15 : a.M) : a.N;
    auto rsrc_of = [&](int m0, int n0) {
        const int r0 = grp == 0 ? m0 : n0;
        const size_t bytes = (size_t)(rows - r0) * ldb;
        return buf_rsrc(src + (size_t)r0 * ldb, (unsigned)(bytes < 0xFFFFFFFFu ? bytes : 0xFFFFFFFFu));
    };
    const int lr = lane >> 3, chunk = (lane & 7) ^ lr;
    unsigned voff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int pc = 8 * (i >> 1) + 2 * wc + (i & 1);
        voff[i] = oblk ? (unsigned)((pc >> 1) * 16 * ldb + (pc & 1) * 1024 + lane * 16)
                       : (unsigned)((pc * 8 + lr) * ldb + chunk * 16);
    }
    const int kstride = oblk ? 2048 : 128;  // bytes per k-tile along a row (block)
    const int opbase = grp == 0 ? 0 : A_BYTES;

    int m0, n0, mn = 0, nn = 0;
    tile(0, m0, n0);  // the launcher sizes the grid <= ntiles
    bool has_next = tile(1, mn, nn);
    i32x4_t rs_c = rsrc_of(m0, n0), rs_n = has_next ? rsrc_of(mn, nn) : rs_c;
    // k-tile j of the current tile's frame (j >= nk: k-tile j - nk of the next tile)
    auto issue = [&](int part, int j) {
        i32x4_t r = rs_c;
        int kk = j;
        if (j >= nk) {
            if (!has_next) return;
            r = rs_n;
            kk = j - nk;
        }
        unsigned char* dst = smem + (j & 1) * STAGE + opbase;  // nk even: the stream's parity
#pragma unroll
        for (int i = 0; i < 2; ++i) blds16(r, voff[2 * part + i], kk * kstride, dst + (8 * part + 2 * wc + i) * 1024);
    };
    f32x4 acc[4][8];
    // prologue (as gemm_pp_kernel)
#pragma unroll
    for (int p = 0; p < 4; ++p) issue(p, 0);
    if (grp == 0) {
        issue(0, 1);
    } else {
        issue(0, 1);
        issue(1, 1);
    }
    // the bias vector -> LDS (ordinary loads: the compiler drains vmcnt before the LDS writes,
    // which only waits for the prologue pieces a little early)
    for (int i = tid; i < a.N; i += 512) colv[i] = a.bias ? a.bias[i] : 0.f;
    if (grp == 0) vm_wait<2>(); else vm_wait<4>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger

    const int lrow = lane & 15, lsw = lane & 7, lg = lane >> 4;
    // W fragments: swizzled row-major image, or (BLKW) chunk-major 16-row blocks
    const int woff = BLKW ? A_BYTES + wc * 64 * 128 + lrow * 16 : A_BYTES + (wc * 64 + lrow) * 128;
    const int s0 = ((0 | lg) ^ lsw) << 4, s1 = ((4 | lg) ^ lsw) << 4;  // swizzled row-major chunks
    const int c0 = BLKW ? lg << 8 : s0, c1 = BLKW ? (4 | lg) << 8 : s1;
    // A fragments: swizzled row-major image, or (blk_a) chunk-major 16-row blocks
    const int aoff = BLKA ? grp * 128 * 128 + lrow * 16 : (grp * 128 + lrow) * 128;
    const int a0 = BLKA ? lg << 8 : s0, a1 = BLKA ? (4 | lg) << 8 : s1;
    vec8 af[4][2], wf[4][2];
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};

    // one k-tile (4 phases); Z: the tile's first k-tile (k-half 0 MFMAs start from zero)
#define MFMA_OR_SINK(C, Wf, Af, ZERO, S, I) C = T::mfma16(Wf, Af, (ZERO) ? zero : C)
    auto ktile = [&](const int kt, const unsigned char* st, auto Zc) {
        constexpr bool Z = decltype(Zc)::value;
        const bool more = kt + 2 < nk || has_next;
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            wf[f][0] = *(const vec8*)(st + woff + f * 2048 + c0);
            wf[f][1] = *(const vec8*)(st + woff + f * 2048 + c1);
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            af[f][0] = *(const vec8*)(st + aoff + f * 2048 + a0);
            af[f][1] = *(const vec8*)(st + aoff + f * 2048 + a1);
        }
        if (grp == 0) issue(1, kt + 1); else issue(2, kt + 1);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int fn = 0; fn < 2; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
                    MFMA_OR_SINK(acc[fn][fm], wf[fn][s], af[fm][s], Z && s == 0, s, fn * 4 + fm);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int f = 2; f < 4; ++f) {
            wf[f][0] = *(const vec8*)(st + woff + f * 2048 + c0);
            wf[f][1] = *(const vec8*)(st + woff + f * 2048 + c1);
        }
        if (grp == 0) issue(2, kt + 1); else issue(3, kt + 1);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int fn = 2; fn < 4; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
                    MFMA_OR_SINK(acc[fn][fm], wf[fn][s], af[fm][s], Z && s == 0, s, fn * 4 + fm);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            af[f][0] = *(const vec8*)(st + aoff + (f + 4) * 2048 + a0);
            af[f][1] = *(const vec8*)(st + aoff + (f + 4) * 2048 + a1);
        }
        if (grp == 0) issue(3, kt + 1); else issue(0, kt + 2);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int fn = 2; fn < 4; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
                    MFMA_OR_SINK(acc[fn][fm + 4], wf[fn][s], af[fm][s], Z && s == 0, s, fn * 4 + fm);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        if (grp == 0) {
            issue(0, kt + 2);
        } else {
            issue(1, kt + 2);
            if (more) vm_wait<4>(); else vm_wait<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int fn = 0; fn < 2; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
                    MFMA_OR_SINK(acc[fn][fm + 4], wf[fn][s], af[fm][s], Z && s == 0, s, fn * 4 + fm);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (grp == 0) {
            if (more) vm_wait<2>(); else vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();
    };

#undef MFMA_OR_SINK
    constexpr bool GELU = EPI == EPI_GELU;
    unsigned char* const Cb = (unsigned char*)a.C;
    for (int i = 1;; ++i) {
        ktile(0, smem, std::true_type{});
        ktile(1, smem + STAGE, std::false_type{});
        for (int kt = 2; kt < nk; kt += 2) {
            ktile(kt, smem, std::false_type{});
            ktile(kt + 1, smem + STAGE, std::false_type{});
        }
        // epilogue of this tile: the other group is in its MFMA segment meanwhile. The lane's 16
        // bias values come from LDS by inline-asm reads: a plain LDS read here makes hipcc drain
        // vmcnt(0) first (the next tile's staging DMA may alias it, as far as it knows)
        const int n = n0 + wc * 64 + 16 * lg;
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
            const int m = m0 + grp * 128 + fm * 16 + lrow;
            float v[16];
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) v[4 * f + rr] = acc[f][fm][rr] + bv[f][rr];
            if constexpr (GELU) {
#pragma unroll
                for (int q = 0; q < 16; ++q) v[q] = quick_gelu(v[q]);
            }
            if (m < a.M) {
                // blocked C (blk_c): the quarter-wave's 16 rows x 16 B are 256 contiguous bytes
                const size_t off = a.blk_c ? blk16_off(m, n, a.ldc) : ((size_t)m * a.ldc + n) * 2;
                const size_t off2 = a.blk_c ? off + 256 : off + 16;
                const u32x4 w0 = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
                const u32x4 w1 = {pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]), pack2<T>(v[12], v[13]),
                                  pack2<T>(v[14], v[15])};
                if constexpr (NT) {  // non-temporal: no L2 allocation for the output (A/B, §5.8)
                    __builtin_nontemporal_store(w0, (u32x4*)(Cb + off));
                    __builtin_nontemporal_store(w1, (u32x4*)(Cb + off2));
                } else {
                    cstore16<PP_AUX_ST>(Cb, off, __builtin_bit_cast(uint4, w0));
                    cstore16<PP_AUX_ST>(Cb, off2, __builtin_bit_cast(uint4, w1));
                }
            }
        }
        if (!has_next) break;
        m0 = mn;
        n0 = nn;
        rs_c = rs_n;
        has_next = tile(i + 1, mn, nn);
        if (has_next) rs_n = rsrc_of(mn, nn);
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
}

template <typename T, bool NT>
static int launch_ppp_t(hipStream_t s, int epi, const GemmArgs& a) {
    const int ncu = a.ncu > 0 ? a.ncu : 256;
    const int ntiles = ((a.M + 255) / 256) * (a.N / 256);
    const int grid = ntiles < ncu ? ntiles : ncu;
    if (a.blk_a) {  // blocked A: c_proj's u, or h in the 16-row blocked layout (QKV / c_fc)
        if (epi == EPI_STORE) {
            if (a.blk_w) gemm_ppp_kernel<T, EPI_STORE, NT, true, true><<<grid, 512, 0, s>>>(a, ntiles);
            else gemm_ppp_kernel<T, EPI_STORE, NT, true><<<grid, 512, 0, s>>>(a, ntiles);
            return 0;
        }
        if (epi == EPI_GELU) {
            if (a.blk_w) gemm_ppp_kernel<T, EPI_GELU, NT, true, true><<<grid, 512, 0, s>>>(a, ntiles);
            else gemm_ppp_kernel<T, EPI_GELU, NT, true><<<grid, 512, 0, s>>>(a, ntiles);
            return 0;
        }
        return -1;
    }
    if (a.blk_w) {  // blocked W
        if (epi == EPI_STORE) { gemm_ppp_kernel<T, EPI_STORE, NT, false, true><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
        if (epi == EPI_GELU) { gemm_ppp_kernel<T, EPI_GELU, NT, false, true><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
        return -1;
    }
    if (epi == EPI_STORE) { gemm_ppp_kernel<T, EPI_STORE, NT><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_GELU) { gemm_ppp_kernel<T, EPI_GELU, NT><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    return -1;
}

template <typename T, bool BLKW, bool NT, int BM = 256>
static int launch_p32_t(hipStream_t s, int epi, const GemmArgs& a, bool balanced = false) {
    if (a.K % 128 || a.K < 256) return -1;  // whole groups of four 32-deep k-steps, >= 2 groups
    if (a.N > (BM <= 256 ? 8192 : 4096)) return -1;  // the bias vector's LDS room (gemm_p32_kernel)
    if ((size_t)(a.M + 15) * a.ldc * 2 >= 0xFFFFFFF0u) return -1;  // C offsets are 32-bit (gemm_p32.h rs_out)
    const int ncu = a.ncu > 0 ? a.ncu : 256;
    const int ntiles = ((a.M + BM - 1) / BM) * (a.N / 256);
    const int per = (ntiles + ncu - 1) / ncu;
    const int grid = balanced ? (ntiles + per - 1) / per : ntiles < ncu ? ntiles : ncu;
    if (a.blk_a) {  // blocked A: c_proj's u, or h in the 16-row blocked layout (QKV / c_fc)
        if (epi == EPI_STORE) { gemm_p32_kernel<T, EPI_STORE, true, BLKW, NT, BM><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
        if (epi == EPI_GELU) { gemm_p32_kernel<T, EPI_GELU, true, BLKW, NT, BM><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
        return -1;
    }
    if (epi == EPI_STORE) { gemm_p32_kernel<T, EPI_STORE, false, BLKW, NT, BM><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_GELU) { gemm_p32_kernel<T, EPI_GELU, false, BLKW, NT, BM><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    return -1;
}

template <typename T>
static int launch_p32(hipStream_t s, int epi, const GemmArgs& a, bool nt, bool bal = false) {
    if (nt) return a.blk_w ? launch_p32_t<T, true, true>(s, epi, a, bal) : launch_p32_t<T, false, true>(s, epi, a, bal);
    return a.blk_w ? launch_p32_t<T, true, false>(s, epi, a, bal) : launch_p32_t<T, false, false>(s, epi, a, bal);
}

// variant 77: 320 x 256 tiles on a balanced grid (c_fc at B/32 bs 256: 480 tiles on 240
// workgroups x 2, against 600 256 x 256 tiles on 200 x 3: 17 % fewer MACs and 25 % fewer staged
// bytes on the busiest CU)
template <typename T>
static int launch_p32_320(hipStream_t s, int epi, const GemmArgs& a) {
    return a.blk_w ? launch_p32_t<T, true, false, 320>(s, epi, a, true) : launch_p32_t<T, false, false, 320>(s, epi, a, true);
}

// variant 79: 192 x 256 tiles on a balanced grid, for the N = 768 roles (out_proj, c_proj at
// B/32 bs 256: 67 x 3 = 201 tiles, one per workgroup): one workgroup stages its A rows once for
// 256 columns, where two 160 x 128 workgroups on a CU stage theirs twice (22 % fewer staged bytes
// per CU than variant 82)
template <typename T>
static int launch_p32_192(hipStream_t s, int epi, const GemmArgs& a) {
    return a.blk_w ? launch_p32_t<T, true, false, 192>(s, epi, a, true) : launch_p32_t<T, false, false, 192>(s, epi, a, true);
}

// variant 62: persistent ping-pong (direct stores; 1-D XCD maps only, N <= 8192); 63: 62 with
// non-temporal stores (the large-M roles of B/16 and L/14@336); 72: the 32-deep-k-step
// persistent tile of gemm_p32.h; 74: 72 with non-temporal stores; 75: 72 on a balanced grid (600
// tiles on 200 workgroups x 3, as hipBLASLt sizes c_fc; tuning fc_variant). GemmArgs.blk_w: W
// in the 16-row blocked layout, every staged k-tile of a 16-row block one contiguous run.
int launch_gemm_pp(hipStream_t s, int dtype, int epi, const GemmArgs& a, int variant) {
    if (a.N % 256 || a.K % 128 || a.K < 128 || a.ksplit > 1) return -1;
    if (a.N > 8192 || xcd_split_n(a.N / 256, a.xcd_n)) return -1;
    if (variant == 62) return dtype == 2 ? launch_ppp_t<F16, false>(s, epi, a) : launch_ppp_t<BF16, false>(s, epi, a);
    if (variant == 72 || variant == 74)
        return dtype == 2 ? launch_p32<F16>(s, epi, a, variant == 74) : launch_p32<BF16>(s, epi, a, variant == 74);
    if (variant == 75)  // 72 on the fewest workgroups with the same tiles per workgroup (the B/32 bs-256 c_fc)
        return dtype == 2 ? launch_p32<F16>(s, epi, a, false, true) : launch_p32<BF16>(s, epi, a, false, true);
    if (variant == 77)  // 320 x 256 tiles, balanced grid
        return dtype == 2 ? launch_p32_320<F16>(s, epi, a) : launch_p32_320<BF16>(s, epi, a);
    if (variant == 79)  // 192 x 256 tiles, balanced grid
        return dtype == 2 ? launch_p32_192<F16>(s, epi, a) : launch_p32_192<BF16>(s, epi, a);
    return -1;
}

}  // namespace clipvit
