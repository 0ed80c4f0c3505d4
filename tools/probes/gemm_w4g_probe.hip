// PROBE (not built into the library): persistent 256x256 MFMA GEMM with ONE wave per SIMD and
// register-staged operands (r05 variant 76, second form). Bit-identical to variant 8, and slower
// than both the LDS-DMA form (gemm_w4_probe.hip) and variant 72 (profiles/r05/w4_probe.txt). To
// re-measure: restore the variant 76 / 77 routing (commit 1a6b0fe) and build this file without
// --amdgpu-mfma-vgpr-form (its 256 accumulators per lane must be AGPRs).
//
//   C[M, N] = A[M, K] @ W[N, K]^T + bias   (16-bit C; QuickGELU for c_fc)
//
// Against gemm_p32.h (variant 72): four waves, each a 128 x 128 sub-tile (64 MFMAs per 32-deep
// k-step), and the operands are staged global -> VGPR -> LDS (buffer_load_dwordx4 + ds_write_b128,
// as the vendor library's MT256x256x64 kernel does for these shapes) instead of LDS-DMA. A wave
// loads k-step t + 3 into registers, writes k-step t + 2 into LDS, and reads the fragments of
// k-step t + 1 while its MFMAs run k-step t; two 32 KB LDS stages. Arithmetic: accumulate from 0,
// then + bias and QuickGELU in the epilogue, exactly as variant 72 / 62 / the pipelined tiles.
#include <type_traits>

#include "common.h"

namespace clipvit {

__device__ u32x4 w4_buffer_load16(i32x4_t rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");

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
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE + 8192 * 4];  // 96 KB
    const float* const colv = (const float*)(smem + 2 * STAGE);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int nM = (a.M + BM - 1) / BM, nN = a.N / BN;
    const int G = gridDim.x;
    const size_t ldb = (size_t)a.K * 2;
    const int nk = a.K >> 5;  // 32-deep k-steps per tile, even, >= 4

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
    const i32x4_t rs_none = buf_rsrc(srcA, 0u);  // no next tile: loads return zeros
    // piece i of this wave = 16 rows 16 p .. 16 p + 15 of each panel, p = 4 wave + i; lane l
    // carries 16 B that land at byte 16 l of the piece (the LDS image of gemm_p32.h)
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

    u32x4 X[2][8];  // the staged pieces of a k-step: A 0-3, W 4-7 (buffer = step & 1)
    auto load_piece = [&](auto bc, const i32x4_t& rA, const i32x4_t& rW, int kk, auto ic) {
        constexpr int B = decltype(bc)::value, I = decltype(ic)::value;
        if constexpr (I < 4) X[B][I] = w4_buffer_load16(rA, (int)voffA[I], koff(BLKA, kk), 0);
        else X[B][I] = w4_buffer_load16(rW, (int)voffW[I - 4], koff(BLKW, kk), 0);
    };
    unsigned char* const wbase = smem + 4 * wave * 1024 + lane * 16;
    auto write_piece = [&](auto bc, auto stc, auto ic) {
        constexpr int B = decltype(bc)::value, ST = decltype(stc)::value, I = decltype(ic)::value;
        *(u32x4*)(wbase + ST * STAGE + (I < 4 ? 0 : A_ST) + (I & 3) * 1024) = X[B][I];
    };

    // fragment addresses: lane (row lrow of a 16-row fragment, k-chunk lg)
    const int lrow = lane & 15, lg = lane >> 4;
    const int swz = ((lg ^ ((lrow >> 2) & 2)) << 4);
    const int aoff = BLKA ? (wm * 8) * 1024 + lg * 256 + lrow * 16 : (wm * 128 + lrow) * 64 + swz;
    const int woff = BLKW ? A_ST + (wn * 8) * 1024 + lg * 256 + lrow * 16 : A_ST + (wn * 128 + lrow) * 64 + swz;
    const unsigned char* const a_rd = smem + aoff;
    const unsigned char* const w_rd = smem + woff;
    vec8 af[2][8], wf[2][8];
    f32x4 acc[8][8];
    // read q (0..15) of stage ST into fragment buffer B: W fragments 0-7, then A fragments 0-7
    auto read_q = [&](auto stc, auto bc, auto qc) {
        constexpr int ST = decltype(stc)::value, B = decltype(bc)::value, Q = decltype(qc)::value;
        if constexpr (Q < 8) wf[B][Q] = *(const vec8*)(w_rd + ST * STAGE + Q * 1024);
        else af[B][Q - 8] = *(const vec8*)(a_rd + ST * STAGE + (Q - 8) * 1024);
    };
    auto bar = [&] {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes and reads done
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
#pragma unroll
            for (int f = 0; f < 4; ++f) bv[f] = *(const f32x4*)(colv + n + 4 * f);
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
            }
        }
    };
    // iteration j (P = j & 1): load k-step j + 3 (buffer P ^ 1; NXT: it belongs to the next tile,
    // kk its step there), write k-step j + 2 (buffer P) into stage P, read k-step j + 1 (stage
    // P ^ 1) into fragment buffer P ^ 1 while the MFMAs run k-step j on buffer P. FIRST: j == 0
    // (accumulators from 0); EP: the previous tile's epilogue goes before this step's MFMAs.
    auto iter = [&](int kk_load, auto pc, auto nxt, auto first, auto ep, bool have_prev, int pm0, int pn0) {
        constexpr int P = decltype(pc)::value;
        constexpr bool FIRST = decltype(first)::value, EP = decltype(ep)::value;
        using PS = std::integral_constant<int, P>;
        using NS = std::integral_constant<int, P ^ 1>;
        const i32x4_t& rA = decltype(nxt)::value ? rA_n : rA_c;
        const i32x4_t& rW = decltype(nxt)::value ? rW_n : rW_c;
        if constexpr (EP) {
            w4_static_for([&](auto ic) { write_piece(PS{}, PS{}, ic); }, std::make_integer_sequence<int, 8>{});
            w4_static_for([&](auto ic) { load_piece(NS{}, rA, rW, kk_load, ic); }, std::make_integer_sequence<int, 8>{});
            if (have_prev) epilogue(pm0, pn0);
        }
        __builtin_amdgcn_sched_barrier(0);
        w4_static_for(
            [&](auto qc) {
                constexpr int Q = decltype(qc)::value;
                if constexpr (!EP) {
                    if constexpr ((Q & 1) == 0) write_piece(PS{}, PS{}, std::integral_constant<int, Q / 2>{});
                    else load_piece(NS{}, rA, rW, kk_load, std::integral_constant<int, Q / 2>{});
                }
                read_q(NS{}, NS{}, qc);
                constexpr int fn0 = (Q & 1) * 4, fm = Q >> 1;  // (fn 0-3 | 4-7) x one A fragment
#pragma unroll
                for (int fn = fn0; fn < fn0 + 4; ++fn)
                    acc[fn][fm] = T::mfma16(wf[P][fn], af[P][fm], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[fn][fm]);
                __builtin_amdgcn_sched_barrier(0);
            },
            std::make_integer_sequence<int, 16>{});
        bar();
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    // prologue: k-steps 0 and 1 into the stages, k-step 2 into registers (buffer 0), the bias
    // vector of the whole GEMM into LDS, the fragments of k-step 0
    w4_static_for([&](auto ic) { load_piece(I0{}, rA_c, rW_c, 0, ic); }, std::make_integer_sequence<int, 8>{});
    w4_static_for([&](auto ic) { load_piece(I1{}, rA_c, rW_c, 1, ic); }, std::make_integer_sequence<int, 8>{});
    for (int i = wave * 64 + lane; i < a.N; i += 256) ((float*)colv)[i] = a.bias ? a.bias[i] : 0.f;
    w4_static_for([&](auto ic) { write_piece(I0{}, I0{}, ic); }, std::make_integer_sequence<int, 8>{});
    w4_static_for([&](auto ic) { write_piece(I1{}, I1{}, ic); }, std::make_integer_sequence<int, 8>{});
    w4_static_for([&](auto ic) { load_piece(I0{}, rA_c, rW_c, 2, ic); }, std::make_integer_sequence<int, 8>{});
    bar();
    w4_static_for([&](auto qc) { read_q(I0{}, I0{}, qc); }, std::make_integer_sequence<int, 16>{});
    bar();  // every wave's reads of stage 0 are done before iteration 0 refills it
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
        for (int m = 0; m < 8; ++m) acc[f][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    int pm0 = 0, pn0 = 0;
    for (int i = 1;; ++i) {
        const bool have_prev = i > 1;
        iter(3, I0{}, F_{}, T_{}, T_{}, have_prev, pm0, pn0);
        iter(4, I1{}, F_{}, F_{}, F_{}, false, 0, 0);
        for (int kt = 2; kt < nk - 4; kt += 2) {
            iter(kt + 3, I0{}, F_{}, F_{}, F_{}, false, 0, 0);
            iter(kt + 4, I1{}, F_{}, F_{}, F_{}, false, 0, 0);
        }
        // last four: loads of k-step nk - 1, then the next tile's k-steps 0, 1, 2; the last
        // iteration reads the next tile's k-step 0 (stage 0)
        iter(nk - 1, I0{}, F_{}, F_{}, F_{}, false, 0, 0);
        iter(0, I1{}, T_{}, F_{}, F_{}, false, 0, 0);
        iter(1, I0{}, T_{}, F_{}, F_{}, false, 0, 0);
        iter(2, I1{}, T_{}, F_{}, F_{}, false, 0, 0);
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
}

// variant 76 / 77 (non-temporal stores). The grid is the fewest workgroups that keep the
// per-workgroup tile count of a full-chip grid (600 tiles on 256 CUs: 3 per workgroup either
// way, so 200 workgroups), as the vendor library sizes its grid.
template <typename T, bool BLKW, bool NT>
static int launch_w4_t(hipStream_t s, int epi, const GemmArgs& a) {
    if (a.K % 64 || a.K < 256) return -1;  // an even number of 32-deep k-steps, >= 8
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
