// PROBE (not built into the library): persistent 256x256 MFMA GEMM with ONE wave per SIMD (r05
// variants 76 / 77). Bit-identical to variant 8 on the race screen, and 5-15 % slower than
// variant 72 on every measured shape (profiles/r05/w4_probe.txt), so it was removed from the
// build. To re-measure it: restore the variant 76 / 77 routing of launch_gemm_pp (git history),
// compile this file without --amdgpu-mfma-vgpr-form (its 256 accumulators per lane must be
// AGPRs) and link it with the library objects.
//
//   C[M, N] = A[M, K] @ W[N, K]^T + bias   (16-bit C; QuickGELU for c_fc)
//
// Why: the 8-wave ping-pong tiles (62 / 72) give each wave a 128 x 64 sub-tile, so every
// 32-deep k-step reads (128 + 64) x 64 B of fragments per wave from LDS: 96 KB per CU for the
// 32 KB staged. Their partner-wave overlap was measured nearly serial (profiles/
// r05_gemm_timeline.md §4). The vendor library's kernel for these shapes
// (hipBLASLt "MT256x256x64", profiles/r05/blas_yardstick.md) runs 256 threads per 256 x 256 tile
// and is 8-12 % faster per tile on c_fc. Here four waves each own a 128 x 128 sub-tile
// (2 x 2 waves): 64 KB of fragment reads per k-step, 64 MFMAs per wave per k-step, and one
// wave interleaves its own fragment reads for k-step t + 1 and its share of the LDS-DMA staging
// of k-step t + 3 with the MFMAs of k-step t. The accumulators (64 x f32x4 = 256 per lane) live
// in AGPRs (512-register budget at one wave per SIMD).
//
// Staging and LDS image: gemm_p32.h's (four 32 KB stages of 32-deep k-steps, the same swizzle
// and the same 16-row blocked layouts for A / W), with 8 pieces of 1 KB per wave per k-step (4 of
// A, 4 of W). Arithmetic: the accumulators start at 0 and the epilogue adds the bias and applies
// QuickGELU exactly as gemm_p32.h / variant 62 / the pipelined tiles, so every tile gives the
// same bits.
//
// Schedule (iteration j of a tile = k-step j's MFMAs):
//   issue DMA of k-step j + 3 (stage (j + 3) & 3, last read in iteration j - 2)
//   [j == 0: the previous tile's epilogue: bias + activation + stores]
//   reads of k-step j + 1 into fragment buffer (j + 1) & 1, interleaved with the 64 MFMAs of
//   k-step j on buffer j & 1
//   lgkmcnt(0); vmcnt: the pieces of k-step j + 2 landed; barrier
#include <type_traits>

#include "common.h"

// schedule knobs (probe builds: tools/r05_runs.sh w4_knobs)
#ifndef W4_FRONT
#define W4_FRONT 0  // 1: a k-step's 8 staging pieces issued before its MFMAs, not interleaved
#endif
#ifndef W4_PRIO
#define W4_PRIO 1  // s_setprio 1 around the MFMA stream
#endif

namespace clipvit {

// f(integral_constant<int, Q>) for Q = 0 .. sizeof...(Q) - 1, in order (compile-time indices)
template <typename F, int... Q>
__device__ __forceinline__ void w4_static_for(F&& f, std::integer_sequence<int, Q...>) {
    (f(std::integral_constant<int, Q>{}), ...);
}

template <typename T, int EPI, bool BLKA, bool BLKW, bool NT>
__global__ __launch_bounds__(256, 1) void gemm_w4_kernel(GemmArgs a, int ntiles) {
    typedef typename T::vec8 vec8;
    constexpr int BM = 256, BN = 256;
    constexpr int A_ST = BM * 64, STAGE = (BM + BN) * 64;  // 16 KB + 16 KB
    constexpr bool GELU = EPI == EPI_GELU;
    __shared__ __attribute__((aligned(16))) unsigned char smem[4 * STAGE + 8192 * 4];  // 160 KB
    const float* const colv = (const float*)(smem + 4 * STAGE);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int nM = (a.M + BM - 1) / BM, nN = a.N / BN;
    const int G = gridDim.x;
    const size_t ldb = (size_t)a.K * 2;
    const int nk = a.K >> 5;  // 32-deep k-steps per tile, a multiple of 4, >= 8

    auto tile = [&](int i, int& m0, int& n0) {
        const int L = blockIdx.x + i * G;
        if (L >= ntiles) return false;
        int mt, nt;
        tile_of_block(L, nM, nN, a.xcd_n, mt, nt);
        m0 = mt * BM;
        n0 = nt * BN;
        return true;
    };
    const unsigned char* const srcA = (const unsigned char*)a.A;
    const unsigned char* const srcW = (const unsigned char*)a.W;
    const int rowsA = BLKA ? (a.M + 15) & ~15 : a.M;
    auto rsrc = [&](const unsigned char* src, int rows, int r0) {
        const size_t bytes = (size_t)(rows - r0) * ldb;
        return buf_rsrc(src + (size_t)r0 * ldb, (unsigned)(bytes < 0xFFFFFFFFu ? bytes : 0xFFFFFFFFu));
    };
    const i32x4_t rs_none = buf_rsrc(srcA, 0u);  // no next tile: reads return zeros
    // piece i of this wave = 16 rows 16 p .. 16 p + 15 of each panel, p = 4 wave + i
    unsigned voffA[4], voffW[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int p = 4 * wave + i;
        const int r = lane >> 2, c = (lane & 3) ^ ((lane >> 4) & 2);
        const unsigned blk = (unsigned)((size_t)p * 16 * ldb + lane * 16);
        const unsigned rm = (unsigned)((16 * p + r) * ldb + c * 16);
        voffA[i] = BLKA ? blk : rm;
        voffW[i] = BLKW ? blk : rm;
    }
    auto koff = [](bool blk, int kk) { return blk ? (kk >> 1) * 2048 + (kk & 1) * 1024 : kk * 64; };
    using T_ = std::true_type;
    using F_ = std::false_type;

    int m0, n0, mn = 0, nn = 0;
    tile(0, m0, n0);
    bool has_next = tile(1, mn, nn);
    i32x4_t rA_c = rsrc(srcA, rowsA, m0), rW_c = rsrc(srcW, a.N, n0);
    i32x4_t rA_n = has_next ? rsrc(srcA, rowsA, mn) : rs_none, rW_n = has_next ? rsrc(srcW, a.N, nn) : rs_none;

    // DMA piece i (0..7: A pieces 0-3, W pieces 4-7) of k-step kk into stage st
    auto piece = [&](const i32x4_t& rA, const i32x4_t& rW, int kk, int st, int i) {
        unsigned char* dst = smem + st * STAGE + 4 * wave * 1024 + (i & 3) * 1024;
        if (i < 4) blds16(rA, voffA[i & 3], koff(BLKA, kk), dst);
        else blds16(rW, voffW[i & 3], koff(BLKW, kk), dst + A_ST);
    };

    // fragment addresses: lane (row lrow of a 16-row fragment, k-chunk lg)
    const int lrow = lane & 15, lg = lane >> 4;
    const int swz = ((lg ^ ((lrow >> 2) & 2)) << 4);
    const int aoff = BLKA ? (wm * 8) * 1024 + lg * 256 + lrow * 16 : (wm * 128 + lrow) * 64 + swz;
    const int woff = BLKW ? A_ST + (wn * 8) * 1024 + lg * 256 + lrow * 16 : A_ST + (wn * 128 + lrow) * 64 + swz;
    // fragment reads: plain LDS loads (hipcc tracks them and places the lgkmcnt waits before the
    // MFMAs that use them; an asynchronous inline-asm read would let the register allocator copy
    // or spill the destination before the data lands) off two base pointers per operand (stages
    // 0 / 1, and 2 / 3 64 KB up), so every offset is a ds_read immediate
    const unsigned char* a_lo = smem + aoff;
    const unsigned char* w_lo = smem + woff;
    const unsigned char* a_hi = a_lo + 65536;
    const unsigned char* w_hi = w_lo + 65536;
    vec8 af[2][8], wf[2][8];
    f32x4 acc[8][8];
    // read q (0..15) of k-step stage ST into buffer B: W fragments 0-7, then A fragments 0-7
    auto read_q = [&](auto stc, auto bc, auto qc) {
        constexpr int ST = decltype(stc)::value, B = decltype(bc)::value, Q = decltype(qc)::value;
        constexpr int SO = (ST & 1) * STAGE;
        if constexpr (Q < 8) wf[B][Q] = *(const vec8*)((ST >= 2 ? w_hi : w_lo) + SO + Q * 1024);
        else af[B][Q - 8] = *(const vec8*)((ST >= 2 ? a_hi : a_lo) + SO + (Q - 8) * 1024);
    };
    auto bar = [&] {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    unsigned char* const Cb = (unsigned char*)a.C;
    auto epilogue = [&](int pm0, int pn0) {
        int le;  // opaque copy of the lane id: per-row offsets are recomputed, not hoisted
        asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
        const int g = le >> 4;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int n = pn0 + wn * 128 + h * 64 + 16 * g;
            f32x4 bv[4];
            {
                const unsigned ba = (unsigned)(size_t)(LDS_AS const float*)(colv + n);
                asm volatile(
                    "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
                    "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
                    : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
                    : "v"(ba)
                    : "memory");
            }
#pragma unroll
            for (int fm = 0; fm < 8; ++fm) {
                const int m = pm0 + wm * 128 + fm * 16 + (le & 15);
                float v[16];
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) v[4 * f + rr] = acc[4 * h + f][fm][rr] + bv[f][rr];
                if constexpr (GELU) {
#pragma unroll
                    for (int q = 0; q < 16; ++q)  // x sigmoid(1.702 x), as gemm_p32.h
                        v[q] = quick_gelu(v[q]);
                }
                u32x4 w0 = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
                u32x4 w1 = {pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]), pack2<T>(v[12], v[13]), pack2<T>(v[14], v[15])};
                size_t off, off2;
                if (a.blk_c) {
                    off = blk16_off(m, n, a.ldc);
                    off2 = off + 256;
                } else {  // row-major: the permlane32 swap of gemm_p32.h (64 contiguous B per row)
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const auto r = __builtin_amdgcn_permlane32_swap(w0[d], w1[d], false, false);
                        w0[d] = r[0];
                        w1[d] = r[1];
                    }
                    off = ((size_t)m * a.ldc + (n - 16 * g)) * 2 + 32 * (g & 1) + 16 * (g >> 1);
                    off2 = off + 64;
                }
                if (m < a.M) {
                    if constexpr (NT) {
                        __builtin_nontemporal_store(w0, (u32x4*)(Cb + off));
                        __builtin_nontemporal_store(w1, (u32x4*)(Cb + off2));
                    } else {
                        *(u32x4*)(Cb + off) = w0;
                        *(u32x4*)(Cb + off2) = w1;
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    };
    // a workgroup's first tile has no previous one: 32 stores through a zero-length buffer
    // resource (dropped by the range check) keep the vmcnt arithmetic of the epilogue step
    const i32x4_t rs_drop = buf_rsrc(a.C, 0u);
    auto null_stores = [&]() {
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 4; ++i)
            asm volatile(
                "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
                "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
                "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
                "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0"
                :
                : "v"(z), "s"(rs_drop)
                : "memory");
    };
    // iteration j (compile-time stage positions): ST = stage of k-step j + 1 (read), STI = stage
    // of k-step j + 3 (staged), B = fragment buffer of k-step j; NXT = the staged step belongs to
    // the next tile (kk = its step there); FIRST = j == 0 (accumulators start at 0); EP = carries
    // the previous tile's epilogue (vmcnt allowance 8 + 32 stores)
    auto iter = [&](int kk_issue, auto nxt, auto stc, auto stic, auto bc, auto first, auto ep, auto w40,
                    bool have_prev, int pm0, int pn0) {
        constexpr int STI = decltype(stic)::value, B = decltype(bc)::value;
        constexpr bool FIRST = decltype(first)::value, EP = decltype(ep)::value;
        using NB = std::integral_constant<int, B ^ 1>;
        const i32x4_t& rA = decltype(nxt)::value ? rA_n : rA_c;
        const i32x4_t& rW = decltype(nxt)::value ? rW_n : rW_c;
        if constexpr (EP || W4_FRONT) {
#pragma unroll
            for (int i = 0; i < 8; ++i) piece(rA, rW, kk_issue, STI, i);
        }
        if constexpr (EP) {  // the previous tile's epilogue needs every accumulator before this step's MFMAs
            if (have_prev) epilogue(pm0, pn0);
            else null_stores();
        }
        // 16 groups: one fragment read of k-step j + 1 + four MFMAs of k-step j (+ one DMA
        // piece in every other group when the pieces were not issued above)
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (W4_PRIO) __builtin_amdgcn_s_setprio(1);
        w4_static_for(
            [&](auto qc) {
                constexpr int Q = decltype(qc)::value;
                if constexpr (!EP && !W4_FRONT && (Q & 1) == 0) piece(rA, rW, kk_issue, STI, Q >> 1);
                read_q(stc, NB{}, qc);
                constexpr int fn0 = (Q & 1) * 4, fm = Q >> 1;  // (fn 0-3 | 4-7) x one A fragment
#pragma unroll
                for (int fn = fn0; fn < fn0 + 4; ++fn)
                    acc[fn][fm] = T::mfma16(wf[B][fn], af[B][fm], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[fn][fm]);
                __builtin_amdgcn_sched_barrier(0);
            },
            std::make_integer_sequence<int, 16>{});
        if constexpr (W4_PRIO) __builtin_amdgcn_s_setprio(0);
        // the pieces of k-step j + 2 landed: younger are k-step j + 3's 8, and in iterations 0
        // and 1 also the 32 epilogue stores issued in iteration 0 after k-step 3's pieces
        if constexpr (decltype(w40)::value) vm_wait<40>(); else vm_wait<8>();
        bar();
    };
    // prologue: k-steps 0, 1, 2 of the first tile; the bias vector of the whole GEMM -> LDS; the
    // fragments of k-step 0
#pragma unroll
    for (int st = 0; st < 3; ++st)
#pragma unroll
        for (int i = 0; i < 8; ++i) piece(rA_c, rW_c, st, st, i);
    {
        float* cv = (float*)(smem + 4 * STAGE);
        for (int i = wave * 64 + lane; i < a.N; i += 256) cv[i] = a.bias ? a.bias[i] : 0.f;
    }
    vm_wait<0>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    w4_static_for([&](auto qc) { read_q(I0{}, I0{}, qc); }, std::make_integer_sequence<int, 16>{});
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
        for (int m = 0; m < 8; ++m) acc[f][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    int pm0 = 0, pn0 = 0;
    for (int i = 1;; ++i) {
        const bool have_prev = i > 1;
        // iteration j: reads stage (j + 1) & 3, stages (j + 3) & 3, MFMAs on buffer j & 1
        iter(3, F_{}, I1{}, I3{}, I0{}, T_{}, T_{}, T_{}, have_prev, pm0, pn0);
        iter(4, F_{}, I2{}, I0{}, I1{}, F_{}, F_{}, T_{}, false, 0, 0);
        iter(5, F_{}, I3{}, I1{}, I0{}, F_{}, F_{}, F_{}, false, 0, 0);
        iter(6, F_{}, I0{}, I2{}, I1{}, F_{}, F_{}, F_{}, false, 0, 0);
        for (int kt = 4; kt < nk - 4; kt += 4) {
            iter(kt + 3, F_{}, I1{}, I3{}, I0{}, F_{}, F_{}, F_{}, false, 0, 0);
            iter(kt + 4, F_{}, I2{}, I0{}, I1{}, F_{}, F_{}, F_{}, false, 0, 0);
            iter(kt + 5, F_{}, I3{}, I1{}, I0{}, F_{}, F_{}, F_{}, false, 0, 0);
            iter(kt + 6, F_{}, I0{}, I2{}, I1{}, F_{}, F_{}, F_{}, false, 0, 0);
        }
        // last four: k-step nk - 1 staged, then the next tile's k-steps 0, 1, 2; the last
        // iteration reads the next tile's k-step 0 (stage 0)
        iter(nk - 1, F_{}, I1{}, I3{}, I0{}, F_{}, F_{}, F_{}, false, 0, 0);
        iter(0, T_{}, I2{}, I0{}, I1{}, F_{}, F_{}, F_{}, false, 0, 0);
        iter(1, T_{}, I3{}, I1{}, I0{}, F_{}, F_{}, F_{}, false, 0, 0);
        iter(2, T_{}, I0{}, I2{}, I1{}, F_{}, F_{}, F_{}, false, 0, 0);
        pm0 = m0;
        pn0 = n0;
        if (!has_next) break;
        m0 = mn;
        n0 = nn;
        rA_c = rA_n;
        rW_c = rW_n;
        has_next = tile(i + 1, mn, nn);
        rA_n = has_next ? rsrc(srcA, rowsA, mn) : rs_none;
        rW_n = has_next ? rsrc(srcW, a.N, nn) : rs_none;
    }
    epilogue(pm0, pn0);
    vm_wait<0>();
}

// variant 76 / 77 (non-temporal stores). The grid is the fewest
// workgroups that keep the per-workgroup tile count of a full-chip grid (600 tiles on 256 CUs:
// 3 per workgroup either way, so 200 workgroups), as the vendor library sizes its grid.
template <typename T, bool BLKW, bool NT>
static int launch_w4_t(hipStream_t s, int epi, const GemmArgs& a) {
    if (a.K % 128 || a.K < 256) return -1;  // whole groups of four 32-deep k-steps, >= 2 groups
    const int ncu = a.ncu > 0 ? a.ncu : 256;
    const int ntiles = ((a.M + 255) / 256) * (a.N / 256);
    const int per = (ntiles + ncu - 1) / ncu;
    const int grid = (ntiles + per - 1) / per;
    if (a.blk_a) {
        if (epi == EPI_STORE) { gemm_w4_kernel<T, EPI_STORE, true, BLKW, NT><<<grid, 256, 0, s>>>(a, ntiles); return 0; }
        return -1;
    }
    if (epi == EPI_STORE) { gemm_w4_kernel<T, EPI_STORE, false, BLKW, NT><<<grid, 256, 0, s>>>(a, ntiles); return 0; }
    if (epi == EPI_GELU) { gemm_w4_kernel<T, EPI_GELU, false, BLKW, NT><<<grid, 256, 0, s>>>(a, ntiles); return 0; }
    return -1;
}

template <typename T>
static int launch_w4(hipStream_t s, int epi, const GemmArgs& a, bool nt) {
    if (nt) return a.blk_w ? launch_w4_t<T, true, true>(s, epi, a) : launch_w4_t<T, false, true>(s, epi, a);
    return a.blk_w ? launch_w4_t<T, true, false>(s, epi, a) : launch_w4_t<T, false, false>(s, epi, a);
}

int launch_gemm_w4(hipStream_t s, int dtype, int epi, const GemmArgs& a, bool nt) {
    return dtype == 2 ? launch_w4<F16>(s, epi, a, nt) : launch_w4<BF16>(s, epi, a, nt);
}

}  // namespace clipvit
