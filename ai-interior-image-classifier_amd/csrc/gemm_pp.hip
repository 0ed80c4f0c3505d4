// Ping-pong MFMA GEMM: 256x256 tiles, 8 waves in two wave groups staggered by one barrier,
// persistent (one workgroup per CU; variants 62 / 63) and stream-K (65).
//
//   C[M, N] = A[M, K] @ W[N, K]^T + bias (16-bit C; QuickGELU for c_fc)
//
// Same operand conventions as gemm.hip (K-major A and packed W, swapped MFMA operands so a lane
// owns one token and 16 contiguous features, LDS rows of 128 B with 16-B chunk c of row r at
// c ^ (r & 7)), different schedule:
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

namespace clipvit {

#if CLIPVIT_ABLATE == 9 || CLIPVIT_ABLATE == 10
typedef float f32x16 __attribute__((ext_vector_type(16)));
template <typename T>
__device__ __forceinline__ f32x16 mfma32(const typename T::vec8& a, const typename T::vec8& b, const f32x16& c) {
    if constexpr (std::is_same<T, F16>::value) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
#endif

// ---------------------------------------------------------------------------------------
// Persistent form (variant 62): one workgroup per CU walks the tiles blockIdx.x, blockIdx.x + G,
// ... (G = grid size; logical ids through the same bijective XCD remap, so every XCD group
// keeps a contiguous range of the row-major tile order each round). The k-tile stream runs on
// across tile boundaries: the last phases of a tile already stage the next tile's first two
// k-tiles, so a tile's prologue load never stalls the CU, and the finished tile's epilogue
// (bias, QuickGELU, 16-bit stores straight from the accumulators) runs in the first read
// segment of the next tile while the other wave group's MFMAs go on. The bias vector of the
// whole GEMM (N <= 8192) is parked in the 32 KB of LDS beside the two stages.

template <typename T, int EPI, bool NT = false, bool BLKA = false>
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
    const bool ablk = BLKA && grp == 0;
    const int rows = grp == 0 ? (BLKA ? (a.M + 15) & ~15 : a.M) : a.N;
    auto rsrc_of = [&](int m0, int n0) {
#if CLIPVIT_ABLATE == 4 || CLIPVIT_ABLATE == 5 || CLIPVIT_ABLATE == 6
        // diagnostic builds only (tools/exp_l2.sh): every tile stages the first A panel (5), the
        // first W panel (6) or both (4), so those operands stay L2-resident (outputs are garbage)
        if ((CLIPVIT_ABLATE != 6 && grp == 0) || (CLIPVIT_ABLATE != 5 && grp == 1)) m0 = n0 = 0;
#endif
        const int r0 = grp == 0 ? m0 : n0;
        const size_t bytes = (size_t)(rows - r0) * ldb;
        return buf_rsrc(src + (size_t)r0 * ldb, (unsigned)(bytes < 0xFFFFFFFFu ? bytes : 0xFFFFFFFFu));
    };
    const int lr = lane >> 3, chunk = (lane & 7) ^ lr;
    unsigned voff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int pc = 8 * (i >> 1) + 2 * wc + (i & 1);
        voff[i] = ablk ? (unsigned)((pc >> 1) * 16 * ldb + (pc & 1) * 1024 + lane * 16)
                       : (unsigned)((pc * 8 + lr) * ldb + chunk * 16);
    }
    const int kstride = ablk ? 2048 : 128;  // bytes per k-tile along a row (block)
    const int opbase = grp == 0 ? 0 : A_BYTES;

    int m0, n0, mn = 0, nn = 0;
    tile(0, m0, n0);  // the launcher sizes the grid <= ntiles
    bool has_next = tile(1, mn, nn);
    i32x4_t rs_c = rsrc_of(m0, n0), rs_n = has_next ? rsrc_of(mn, nn) : rs_c;
    // k-tile j of the current tile's frame (j >= nk: k-tile j - nk of the next tile)
    auto issue = [&](int part, int j) {
#if CLIPVIT_ABLATE == 7 || CLIPVIT_ABLATE == 10  // diagnostic builds only (tools/exp_l2.sh): no staging after the first two k-tiles
        if (j >= 2) return;
#endif
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
    const int woff = A_BYTES + (wc * 64 + lrow) * 128;
    const int c0 = ((0 | lg) ^ lsw) << 4, c1 = ((4 | lg) ^ lsw) << 4;
    // A fragments: swizzled row-major image, or (blk_a) chunk-major 16-row blocks
    const int aoff = BLKA ? grp * 128 * 128 + lrow * 16 : (grp * 128 + lrow) * 128;
    const int a0 = BLKA ? lg << 8 : c0, a1 = BLKA ? (4 | lg) << 8 : c1;
    vec8 af[4][2], wf[4][2];
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};

    // one k-tile (4 phases); Z: the tile's first k-tile (k-half 0 MFMAs start from zero)
#if CLIPVIT_ABLATE == 8  // diagnostic build only (tools/exp_l2.sh): no MFMAs (fragments kept live)
#define MFMA_OR_SINK(C, Wf, Af, ZERO, S, I) asm volatile("" ::"v"(Wf), "v"(Af))
#elif CLIPVIT_ABLATE == 9 || CLIPVIT_ABLATE == 10
    // diagnostic builds only (tools/exp_l2.sh): every pair of 16x16x32 MFMAs (same FLOPs, same
    // matrix-pipe cycles) replaced by one 32x32x16 MFMA into scratch accumulators (half the MFMA
    // issue slots; outputs are garbage); 10: also no staging after the first two k-tiles
#define MFMA_OR_SINK(C, Wf, Af, ZERO, S, I)                  \
    do {                                                     \
        if ((S) == 0) dacc[(I) & 3] = mfma32<T>(Wf, Af, dacc[(I) & 3]); \
        else asm volatile("" ::"v"(Wf), "v"(Af));           \
    } while (0)
    f32x16 dacc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) dacc[i][j] = 0.f;
#else
#define MFMA_OR_SINK(C, Wf, Af, ZERO, S, I) C = T::mfma16(Wf, Af, (ZERO) ? zero : C)
#endif
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
#if CLIPVIT_ABLATE == 8 || CLIPVIT_ABLATE == 9 || CLIPVIT_ABLATE == 10
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int m = 0; m < 8; ++m) acc[f][m] = zero;
#endif
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
                for (int q = 0; q < 16; ++q) v[q] *= __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v[q]));
            }
#if CLIPVIT_ABLATE == 3  // diagnostic build only: no epilogue stores (values kept live)
            if (m < a.M && a.ldc > (1 << 30)) {
#else
            if (m < a.M) {
#endif
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
                    *(u32x4*)(Cb + off) = w0;
                    *(u32x4*)(Cb + off2) = w1;
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
#if CLIPVIT_ABLATE == 9 || CLIPVIT_ABLATE == 10
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(dacc[i]));
#endif
    if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
}

// ---------------------------------------------------------------------------------------
// Stream-K form (variant 65). The persistent tile's k-tile stream, but each
// workgroup owns an equal contiguous share [b, e) of the GEMM's ntiles * nk k-tile iterations
// (tile-major, tiles in the XCD-aware order of tile_of_block; workgroup positions remapped so the
// workgroups of one XCD hold a contiguous range of that order). A share is cut into jobs: the
// suffix [b % nk, nk) of the tile it starts in (EARLY), whole tiles, and the prefix [0, e % nk)
// of the tile it ends in (LATE). The EARLY part's fp32 accumulators go to a workspace slot
// (sc1 write-through stores, lane-linear, one 32 KB run per wave) and wave w publishes flag w of
// the slot (sc1 store after its vmcnt(0)); the workgroup owning the LATE prefix of that tile
// waits for the flag of its own wave number (sc1 poll: wave w reads only wave w's bytes, the same
// lane <-> element map), loads the partial into its accumulators (sc1 loads) and accumulates the
// prefix k-tiles on top, then runs the ordinary epilogue. Jobs run in the order EARLY, first
// whole tile, LATE, remaining whole tiles, so the partner's EARLY suffix (at most nk - 1
// k-tiles, first in its share) has long finished when LATE starts (after nk + 1 or more).
// Each tile's arithmetic is fixed by the partition: the split tiles add the EARLY partial first,
// then the prefix k-tiles, so a given (M, N, K, grid) is deterministic; other M split elsewhere
// (rounding-level differences, not bit-identical to the one-tile-per-workgroup kernels).
// No deadlock by construction: a LATE job waits only on a higher position's FIRST job, and with a
// bounded wait (~0.1 s): on expiry it writes the error word and uses a zero partial.
__device__ void sk_store4(f32x4 vdata, i32x4_t rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4f32");
__device__ f32x4 sk_load4(i32x4_t rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ unsigned sk_load1(i32x4_t rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.i32");
__device__ void sk_store1(unsigned v, i32x4_t rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.store.i32");
constexpr int SK_SC1 = 16;                      // cache policy: sc1 (agent-coherent write-through / L1 bypass)
constexpr size_t SK_SLOT = 256 * 256 * 4;       // fp32 partial of one 256x256 tile

template <typename T, int EPI>
__global__ __launch_bounds__(512, 1) void gemm_psk_kernel(GemmArgs a, int ntiles) {
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
    const int nk = a.K >> 6;

    // ---- this workgroup's share: position p (XCD-contiguous), k-tile range [b, e)
    int p;
    {
        const int bid = blockIdx.x, q = G >> 3, r = G & 7, x = bid & 7;
        p = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    }
    const long long I = (long long)ntiles * nk;
    const int b = (int)(I * p / G), e = (int)(I * (p + 1) / G);
    const int ks = b % nk, ke = e % nk;
    const int hA = ks > 0, hZ = ke > 0;
    const int tF = (b + nk - 1) / nk, nF = e / nk - tF;
    const int njob = hA + nF + hZ;
    const int L = e - b;  // k-tiles of the share
    // job j -> (tile, first k, count, kind: 0 whole, 1 EARLY, 2 LATE); order A, F0, Z, F1..
    auto job = [&](int j, int& t, int& k0, int& n, int& kind) {
        if (hA && j == 0) { t = b / nk; k0 = ks; n = nk - ks; kind = 1; return; }
        j -= hA;
        if (nF > 0) {
            if (j == 0) { t = tF; k0 = 0; n = nk; kind = 0; return; }
            --j;
        }
        if (hZ && j == 0) { t = e / nk; k0 = 0; n = ke; kind = 2; return; }
        j -= hZ;
        t = tF + 1 + j; k0 = 0; n = nk; kind = 0;
    };

    const unsigned char* src = (const unsigned char*)(grp == 0 ? a.A : a.W);
    const int rows = grp == 0 ? a.M : a.N;
    // tile t -> its (m0, n0) packed as m0 * 65536 + n0 / 256 ... kept as one uniform int
    auto origin = [&](int t) {
        int mt, nt;
        tile_of_block(t, nM, nN, a.xcd_n, mt, nt);
        return mt * 65536 + nt;
    };
    auto rsrc_tile = [&](int o) {
        const int r0 = grp == 0 ? (o >> 16) * BM : (o & 0xffff) * BN;
        const size_t bytes = (size_t)(rows - r0) * ldb;
        return buf_rsrc(src + (size_t)r0 * ldb, (unsigned)(bytes < 0xFFFFFFFFu ? bytes : 0xFFFFFFFFu));
    };
    const int lr = lane >> 3, chunk = (lane & 7) ^ lr;
    unsigned voff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int pc = 8 * (i >> 1) + 2 * wc + (i & 1);
        voff[i] = (unsigned)((pc * 8 + lr) * ldb + chunk * 16);
    }
    const int opbase = grp == 0 ? 0 : A_BYTES;

    // staging lookahead: the current job and the next two (a job has >= 1 k-tile; the stream
    // issues k-tiles s + 1 and s + 2 while k-tile s runs)
    int jc = 0, s0c = 0;  // current job index and its first stream position
    int tc, kc, nc, kindc, t1 = 0, k1 = 0, n1 = 0, kind1 = 0, t2 = 0, k2 = 0, n2 = 0, kind2 = 0;
    job(0, tc, kc, nc, kindc);
    if (njob > 1) job(1, t1, k1, n1, kind1);
    if (njob > 2) job(2, t2, k2, n2, kind2);
    int oc = origin(tc), o1 = njob > 1 ? origin(t1) : oc, o2 = njob > 2 ? origin(t2) : oc;
    i32x4_t rs_c = rsrc_tile(oc), rs_1 = rsrc_tile(o1), rs_2 = rsrc_tile(o2);
    (void)kind1;
    (void)kind2;
    // stream position s2 -> (resource, k); s2 < L
    auto issue = [&](int part, int s2) {
        if (s2 >= L) return;
        int rel = s2 - s0c;
        i32x4_t r = rs_c;
        int kk = kc + rel;
        if (rel >= nc) {
            rel -= nc;
            if (rel < n1) { r = rs_1; kk = k1 + rel; }
            else { r = rs_2; kk = k2 + rel - n1; }
        }
        // the selection is wave-uniform: say so, or hipcc keeps the descriptor in VGPRs and wraps
        // every load in a readfirstlane waterfall loop (cdna_hip_programming.md T20)
        r.x = __builtin_amdgcn_readfirstlane(r.x);
        r.y = __builtin_amdgcn_readfirstlane(r.y);
        r.z = __builtin_amdgcn_readfirstlane(r.z);
        r.w = __builtin_amdgcn_readfirstlane(r.w);
        kk = __builtin_amdgcn_readfirstlane(kk);
        unsigned char* dst = smem + (s2 & 1) * STAGE + opbase;
#pragma unroll
        for (int i = 0; i < 2; ++i) blds16(r, voff[2 * part + i], kk * 128, dst + (8 * part + 2 * wc + i) * 1024);
    };

    f32x4 acc[4][8];
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    unsigned long long* const trace = a.sk_trace ? a.sk_trace + (size_t)p * 8 : nullptr;
    auto stamp = [&](int i) {
        if (trace && wave == 0 && lane == 0 && i < 8) trace[i] = __builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    // prologue: stream k-tile 0 whole, then what the steady state issues before phase q0
#pragma unroll
    for (int q = 0; q < 4; ++q) issue(q, 0);
    if (grp == 0) {
        issue(0, 1);
    } else {
        issue(0, 1);
        issue(1, 1);
    }
    for (int i = tid; i < a.N; i += 512) colv[i] = a.bias ? a.bias[i] : 0.f;
    if (grp == 0) vm_wait<2>(); else vm_wait<4>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger

    const int lrow = lane & 15, lsw = lane & 7, lg = lane >> 4;
    const int aoff = (grp * 128 + lrow) * 128, woff = A_BYTES + (wc * 64 + lrow) * 128;
    const int c0 = ((0 | lg) ^ lsw) << 4, c1 = ((4 | lg) ^ lsw) << 4;
    vec8 af[4][2], wf[4][2];

    // one k-tile (4 phases) at stream position s. A job starts from zeroed accumulators or, LATE,
    // from the loaded partial (acc is defined afresh at the top of every job: not loop-carried).
    auto ktile = [&](const int s, const unsigned char* st) {
        const bool more = s + 2 < L;
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            wf[f][0] = *(const vec8*)(st + woff + f * 2048 + c0);
            wf[f][1] = *(const vec8*)(st + woff + f * 2048 + c1);
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            af[f][0] = *(const vec8*)(st + aoff + f * 2048 + c0);
            af[f][1] = *(const vec8*)(st + aoff + f * 2048 + c1);
        }
        if (grp == 0) issue(1, s + 1); else issue(2, s + 1);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int fn = 0; fn < 2; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
                    acc[fn][fm] = T::mfma16(wf[fn][q], af[fm][q], acc[fn][fm]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int f = 2; f < 4; ++f) {
            wf[f][0] = *(const vec8*)(st + woff + f * 2048 + c0);
            wf[f][1] = *(const vec8*)(st + woff + f * 2048 + c1);
        }
        if (grp == 0) issue(2, s + 1); else issue(3, s + 1);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int fn = 2; fn < 4; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
                    acc[fn][fm] = T::mfma16(wf[fn][q], af[fm][q], acc[fn][fm]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            af[f][0] = *(const vec8*)(st + aoff + (f + 4) * 2048 + c0);
            af[f][1] = *(const vec8*)(st + aoff + (f + 4) * 2048 + c1);
        }
        if (grp == 0) issue(3, s + 1); else issue(0, s + 2);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int fn = 2; fn < 4; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
                    acc[fn][fm + 4] = T::mfma16(wf[fn][q], af[fm][q], acc[fn][fm + 4]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        if (grp == 0) {
            issue(0, s + 2);
        } else {
            issue(1, s + 2);
            if (more) vm_wait<4>(); else vm_wait<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int fn = 0; fn < 2; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
                    acc[fn][fm + 4] = T::mfma16(wf[fn][q], af[fm][q], acc[fn][fm + 4]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (grp == 0) {
            if (more) vm_wait<2>(); else vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();
    };

    constexpr bool GELU = EPI == EPI_GELU;
    unsigned char* const Cb = (unsigned char*)a.C;
    // partial slots: lane-linear, 32 KB per wave; j = 8 f + fm
    const int pvo = wave * 32768 + lane * 16;
    int s = 0;
    for (;;) {
        const int m0 = (oc >> 16) * BM, n0 = (oc & 0xffff) * BN;
        if (kindc == 2) {  // LATE: wait for the partner's EARLY partial (slot p + 1), load it
            const i32x4_t rp = buf_rsrc((const unsigned char*)a.sk_part + (size_t)(p + 1) * SK_SLOT, (unsigned)SK_SLOT);
            const i32x4_t rf = buf_rsrc(a.sk_flag, (unsigned)((G + 1) * 8 * 4));
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            stamp(6);
            bool ok = true;
            while (__builtin_amdgcn_readfirstlane(sk_load1(rf, 0, ((p + 1) * 8 + wave) * 4, SK_SC1)) != a.sk_epoch) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) {  // 0.1 s at 100 MHz
                    ok = false;
                    if (lane == 0) sk_store1(a.sk_epoch, rf, 0, G * 8 * 4, SK_SC1);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int fm = 0; fm < 8; ++fm) acc[f][fm] = ok ? sk_load4(rp, pvo, (8 * f + fm) * 1024, SK_SC1) : zero;
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), visible to the compiler's scoreboard
            stamp(7);
        } else {
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int fm = 0; fm < 8; ++fm) acc[f][fm] = zero;
        }
        for (int i = 0; i < nc; ++i, ++s) ktile(s, smem + (s & 1) * STAGE);
        if (kindc == 1) {  // EARLY: the fp32 partial to slot p, then this wave's flag
            const i32x4_t rp = buf_rsrc((unsigned char*)a.sk_part + (size_t)p * SK_SLOT, (unsigned)SK_SLOT);
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int fm = 0; fm < 8; ++fm) sk_store4(acc[f][fm], rp, pvo, (8 * f + fm) * 1024, SK_SC1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) {
                const i32x4_t rf = buf_rsrc(a.sk_flag, (unsigned)((G + 1) * 8 * 4));
                sk_store1(a.sk_epoch, rf, 0, (p * 8 + wave) * 4, SK_SC1);
            }
        } else {  // whole tile or LATE prefix: the epilogue (as gemm_ppp_kernel, direct stores)
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
                    for (int q = 0; q < 16; ++q) v[q] *= __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v[q]));
                }
                if (m < a.M) {
                    const size_t off = ((size_t)m * a.ldc + n) * 2;
                    const u32x4 w0 = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
                    const u32x4 w1 = {pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]), pack2<T>(v[12], v[13]),
                                      pack2<T>(v[14], v[15])};
                    *(u32x4*)(Cb + off) = w0;
                    *(u32x4*)(Cb + off + 16) = w1;
                }
            }
        }
        stamp(1 + jc);
        if (++jc >= njob) break;
        s0c = s;
        tc = t1; kc = k1; nc = n1; kindc = kind1; rs_c = rs_1; oc = o1;
        t1 = t2; k1 = k2; n1 = n2; kind1 = kind2; rs_1 = rs_2; o1 = o2;
        if (jc + 2 < njob) {
            job(jc + 2, t2, k2, n2, kind2);
            o2 = origin(t2);
            rs_2 = rsrc_tile(o2);
        }
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
}

template <typename T, bool NT>
static int launch_ppp_t(hipStream_t s, int epi, const GemmArgs& a) {
    const int ncu = a.ncu > 0 ? a.ncu : 256;
    const int ntiles = ((a.M + 255) / 256) * (a.N / 256);
    const int grid = ntiles < ncu ? ntiles : ncu;
    if (a.blk_a) {  // blocked A (u): c_proj on the persistent tile (tuning / large-M shapes)
        if (epi == EPI_STORE) { gemm_ppp_kernel<T, EPI_STORE, NT, true><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
        return -1;
    }
    if (epi == EPI_STORE) { gemm_ppp_kernel<T, EPI_STORE, NT><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_GELU) { gemm_ppp_kernel<T, EPI_GELU, NT><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    return -1;
}

template <typename T>
static int launch_psk_t(hipStream_t s, int epi, const GemmArgs& a) {
    const int ncu = a.ncu > 0 ? a.ncu : 256;
    const int ntiles = ((a.M + 255) / 256) * (a.N / 256);
    const int nk = a.K / 64;
    const long long I = (long long)ntiles * nk;
    const int grid = ncu;
    // every share must cover at least one tile's k-tiles (EARLY and LATE then lie in different
    // tiles, and a tile is split between at most two workgroups)
    if (I / grid < nk || !a.sk_part || !a.sk_flag) return launch_ppp_t<T, false>(s, epi, a);  // whole tiles
    if (epi == EPI_STORE) { gemm_psk_kernel<T, EPI_STORE><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_GELU) { gemm_psk_kernel<T, EPI_GELU><<<grid, 512, 0, s>>>(a, ntiles); return 0; }
    return -1;
}

// variant 62: persistent ping-pong (direct stores; 1-D XCD maps only, N <= 8192); 63: 62 with
// non-temporal stores; 65: stream-K (a.sk_part / a.sk_flag workspace; whole tiles where a share
// would be shorter than one tile's k-tiles)
int launch_gemm_pp(hipStream_t s, int dtype, int epi, const GemmArgs& a, int variant) {
    if (a.N % 256 || a.K % 128 || a.K < 128 || a.ksplit > 1) return -1;
    if (a.N > 8192 || xcd_split_n(a.N / 256, a.xcd_n)) return -1;
    if (variant == 65) return dtype == 2 ? launch_psk_t<F16>(s, epi, a) : launch_psk_t<BF16>(s, epi, a);
    if (variant == 63) return dtype == 2 ? launch_ppp_t<F16, true>(s, epi, a) : launch_ppp_t<BF16, true>(s, epi, a);
    if (variant == 62) return dtype == 2 ? launch_ppp_t<F16, false>(s, epi, a) : launch_ppp_t<BF16, false>(s, epi, a);
    return -1;
}

}  // namespace clipvit
