// MX-fp8 form of the persistent 32-deep-k-step GEMM (gemm_p32.h), MX variant 4. Included by
// mx8.hip.
//
//   C[M, N] = dequant(A8)[M, K] @ dequant(W8)[N, K]^T + bias
//   (EPI_STORE: 16-bit row-major C; EPI_GELU_Q8: QuickGELU, then MX-fp8 C with E8M0 block scales)
//
// The schedule, the LDS ring and the counted waits are gemm_p32.h's (two groups of four waves in
// ping-pong, group 0 stages A and group 1 stages W, four stages, the previous tile's epilogue in
// the first read segment of the next). What differs:
//  * the MFMA is v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x e4m3, E8M0 block scales applied in
//    hardware, 2x the 16-bit MFMA rate). A 64-deep fp8 k-step is a 64-byte row, so a stage holds
//    the same bytes as the 16-bit kernel's 32-deep step (32 KB) and the k-step count halves;
//    a wave's segment is 8 MFMAs (its 128 x 64 tile as 4 token blocks x 2 feature blocks of 32)
//    = 512 matrix cycles, as in the 16-bit kernel;
//  * operand lane map (tools/probes/mx32_probe.hip): lane l holds row l & 31 of a 32-row
//    fragment; bytes 0-15 are 16-B chunk h = l >> 5 of the 64-B row (k-block 0) and bytes 16-31
//    chunk h + 2 (k-block 1). The scale of lane r + 32 b applies to row r, k-block b: a lane passes
//    its row's scale dword (the four E8M0 bytes of the 128-deep k-tile) shifted right by 8 h, and
//    the MFMA's opsel 2 (step & 1) picks the byte of this 64-deep half;
//  * LDS image: rows of 64 B, 16-B chunk c of row r at c ^ ((r >> 2) & 3), conflict-free for the
//    32 x 32 fragment reads (each lane-group of ds_read_b128 covers all 64 banks); behind the
//    operands each stage carries the scale dword of every A and W row (2 KB), staged with the
//    pieces by one 4-byte LDS-DMA per wave (5 VMEM issues per wave and k-step);
//  * the swapped-operand accumulator (A operand = W fragment, B operand = tokens) gives lane l
//    token l & 31 and, with the packer's 64-row weight permutation (pack_weight_mx8), the 16
//    contiguous features 16 h .. 16 h + 15 ("run 0") and 32 + 16 h .. ("run 1") of the wave's
//    64-feature slice; an MX output block (32 features) is run r of lanes l and l ^ 32;
//  * epilogue stores are range-checked buffer stores issued unconditionally (rows past M are
//    dropped by the range check), so the store count the waits allow for never varies.
// The fp32 sums are grouped by 64 k per instruction (the 16 x 16 x 128 tiles of variants 1-3
// group by 128): results agree with theirs to fp32 rounding, not bit for bit.
#pragma once
#include <type_traits>

#include "common.h"

namespace clipvit {

typedef int i32x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ void raw_buffer_store_i8(char data, i32x4_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.i8");

template <typename TO, int EPI, bool BLKC, int GRP>
__device__ __forceinline__ void p32mx_body(const GemmArgs& a, int ntiles, unsigned char* smem, int lane, int wc) {
    constexpr int BM = 256, BN = 256;
    constexpr int A_ST = BM * 64, OPS = (BM + BN) * 64, STAGE = OPS + (BM + BN) * 4;  // 34 KB
    constexpr int NP = 4;                                  // 1 KB operand pieces per wave and k-step
    constexpr bool Q8 = EPI == EPI_GELU_Q8;
    constexpr bool F32 = EPI == EPI_F32 || EPI == EPI_F32GELU;  // fp32 C (tests)
    constexpr bool GELU = Q8 || EPI == EPI_F32GELU;
    // epilogue stores per wave: 2 runs x 4 blocks x (2 x 16 B | 16 B + scale byte | 4 x 16 B)
    constexpr int NSTORE = F32 ? 32 : 16;
    constexpr int W_LO = 2 * (NP + 1), W_HI = W_LO + NSTORE;
    const float* const colv = (const float*)(smem + 4 * STAGE);
    const int nM = (a.M + BM - 1) / BM, nN = a.N / BN;
    const int G = gridDim.x;
    const unsigned ldb = (unsigned)a.K, lsc = (unsigned)(a.K >> 5);
    const int nk = a.K >> 6;  // 64-deep k-steps per tile, a multiple of 4, >= 8 (launcher)

    auto tile = [&](int i, int& m0, int& n0) {
        const int L = blockIdx.x + i * G;
        if (L >= ntiles) return false;
        int mt, nt;
        tile_of_block(L, nM, nN, a.xcd_n, mt, nt);
        m0 = mt * BM;
        n0 = nt * BN;
        return true;
    };
    const unsigned char* const src = (const unsigned char*)(GRP == 0 ? a.A : a.W);
    const unsigned char* const ssrc = GRP == 0 ? a.sA : a.sW;
    const int rows = GRP == 0 ? a.M : a.N;
    auto rsrc_of = [&](int m0, int n0) {
        const int r0 = GRP == 0 ? m0 : n0;
        return buf_rsrc(src + (size_t)r0 * ldb, (unsigned)((size_t)(rows - r0) * ldb));
    };
    const i32x4_t rs_none = buf_rsrc(src, 0u);
    const i32x4_t ss_all = buf_rsrc(ssrc, (unsigned)((size_t)rows * lsc));
    const i32x4_t ss_none = buf_rsrc(ssrc, 0u);
    // this wave's scale row = tile row r0 + 64 wc + lane (rows past the operand read 0)
    auto sv_of = [&](int m0, int n0) { return (unsigned)((GRP == 0 ? m0 : n0) + wc * 64 + lane) * lsc; };
    unsigned voff[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int p = NP * wc + i, r = lane >> 2, c = (lane & 3) ^ ((r >> 2) & 3);
        voff[i] = (unsigned)(16 * p + r) * ldb + (unsigned)c * 16u;
    }
    const int opbase = GRP == 0 ? 0 : A_ST;
    const int scbase = OPS + GRP * 1024 + wc * 256;
    auto stage_pieces = [&](const i32x4_t& r, const i32x4_t& sr, unsigned sv, int kk, int st) {
        unsigned char* dst = smem + st * STAGE + opbase + NP * wc * 1024;
#pragma unroll
        for (int i = 0; i < NP; ++i) blds16(r, voff[i], kk * 64, dst + i * 1024);
        raw_buffer_load_lds(sr, (LDS_AS void*)(smem + st * STAGE + scbase), 4, (int)sv, (kk >> 1) * 4, 0, 0);
    };

    int m0, n0, mn = 0, nn = 0;
    tile(0, m0, n0);
    bool has_next = tile(1, mn, nn);
    i32x4_t rs_c = rsrc_of(m0, n0), rs_n = has_next ? rsrc_of(mn, nn) : rs_none;
    i32x4_t ss_n = has_next ? ss_all : ss_none;
    unsigned sv_c = sv_of(m0, n0), sv_n = has_next ? sv_of(mn, nn) : 0u;

    // fragment addresses (lane: row lrow of a 32-row fragment, half h): the two 16-B chunks of
    // the lane's row at chunk h ^ sw and (h ^ sw) ^ 2; bases for stages 0 / 1 and (2 STAGE up)
    // 2 / 3, fragment and stage offsets as immediates below 64 KB
    const int lrow = lane & 31, h = lane >> 5, sw = (lrow >> 2) & 3;
    const int c0 = (h ^ sw) << 4, c1 = ((h ^ sw) ^ 2) << 4;
    const unsigned a_row = (unsigned)(size_t)(LDS_AS unsigned char*)(smem + (GRP * 128 + lrow) * 64);
    const unsigned w_row = (unsigned)(size_t)(LDS_AS unsigned char*)(smem + A_ST + (wc * 64 + lrow) * 64);
    unsigned a0_lo = a_row + c0, a1_lo = a_row + c1, w0_lo = w_row + c0, w1_lo = w_row + c1;
    unsigned a0_hi = a0_lo + 2 * STAGE, a1_hi = a1_lo + 2 * STAGE, w0_hi = w0_lo + 2 * STAGE, w1_hi = w1_lo + 2 * STAGE;
    asm volatile("" : "+v"(a0_lo), "+v"(a1_lo), "+v"(w0_lo), "+v"(w1_lo), "+v"(a0_hi), "+v"(a1_hi), "+v"(w0_hi), "+v"(w1_hi));
    // scale dwords: token rows GRP * 128 + 32 mb + lrow, W rows 64 wc + 32 fb + lrow
    unsigned as_lo = (unsigned)(size_t)(LDS_AS unsigned char*)(smem + OPS + (GRP * 128 + lrow) * 4);
    unsigned ws_lo = (unsigned)(size_t)(LDS_AS unsigned char*)(smem + OPS + 1024 + (wc * 64 + lrow) * 4);
    unsigned as_hi = as_lo + 2 * STAGE, ws_hi = ws_lo + 2 * STAGE;
    asm volatile("" : "+v"(as_lo), "+v"(ws_lo), "+v"(as_hi), "+v"(ws_hi));
    const int hsh = 8 * h;

    i32x4_t af[4][2], wf[2][2];
    int as[4], ws[2];
    f32x16 acc[2][4];

    auto rd = [&](i32x4_t& d, unsigned base, auto imm) {
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(base), "i"(decltype(imm)::value));
    };
    auto rd32 = [&](int& d, unsigned base, auto imm) {
        asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(d) : "v"(base), "i"(decltype(imm)::value));
    };
    auto reads = [&](auto stc) {
        constexpr int ST = decltype(stc)::value, SO = (ST & 1) * STAGE;
        const bool hi = ST >= 2;
        const unsigned wb0 = hi ? w0_hi : w0_lo, wb1 = hi ? w1_hi : w1_lo;
        const unsigned ab0 = hi ? a0_hi : a0_lo, ab1 = hi ? a1_hi : a1_lo;
        const unsigned asb = hi ? as_hi : as_lo, wsb = hi ? ws_hi : ws_lo;
        rd(wf[0][0], wb0, std::integral_constant<int, SO>{});
        rd(wf[0][1], wb1, std::integral_constant<int, SO>{});
        rd(wf[1][0], wb0, std::integral_constant<int, SO + 2048>{});
        rd(wf[1][1], wb1, std::integral_constant<int, SO + 2048>{});
        rd32(ws[0], wsb, std::integral_constant<int, SO>{});
        rd32(ws[1], wsb, std::integral_constant<int, SO + 128>{});
        rd(af[0][0], ab0, std::integral_constant<int, SO>{});
        rd(af[0][1], ab1, std::integral_constant<int, SO>{});
        rd(af[1][0], ab0, std::integral_constant<int, SO + 2048>{});
        rd(af[1][1], ab1, std::integral_constant<int, SO + 2048>{});
        rd(af[2][0], ab0, std::integral_constant<int, SO + 4096>{});
        rd(af[2][1], ab1, std::integral_constant<int, SO + 4096>{});
        rd(af[3][0], ab0, std::integral_constant<int, SO + 6144>{});
        rd(af[3][1], ab1, std::integral_constant<int, SO + 6144>{});
        rd32(as[0], asb, std::integral_constant<int, SO>{});
        rd32(as[1], asb, std::integral_constant<int, SO + 128>{});
        rd32(as[2], asb, std::integral_constant<int, SO + 256>{});
        rd32(as[3], asb, std::integral_constant<int, SO + 384>{});
    };
    auto mfmas = [&](auto first, auto stc) {
        constexpr bool FIRST = decltype(first)::value;
        constexpr int OS = 2 * (decltype(stc)::value & 1);  // byte of the scale dword: this 64-deep half
        const f32x16 zero = {};
        int wsv[2], asv[4];
#pragma unroll
        for (int f = 0; f < 2; ++f) wsv[f] = ws[f] >> hsh;
#pragma unroll
        for (int m = 0; m < 4; ++m) asv[m] = as[m] >> hsh;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int fb = 0; fb < 2; ++fb) {
                const i32x8_t wv = __builtin_shufflevector(wf[fb][0], wf[fb][1], 0, 1, 2, 3, 4, 5, 6, 7);
                const i32x8_t av = __builtin_shufflevector(af[mb][0], af[mb][1], 0, 1, 2, 3, 4, 5, 6, 7);
                acc[fb][mb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                    wv, av, FIRST ? zero : acc[fb][mb], 0, 0, OS, wsv[fb], OS, asv[mb]);
            }
        __builtin_amdgcn_s_setprio(0);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };

    // epilogue C resources: row-major rows >= M fall outside (dropped); blocked u8 keeps its last
    // 16-row block's padding rows (the consumer reads them only into unstored rows)
    const int mpad = (a.M + 15) & ~15;
    const i32x4_t rs_out = buf_rsrc(a.C, (unsigned)((size_t)(Q8 && BLKC ? mpad : a.M) * a.ldc * (Q8 ? 1 : F32 ? 4 : 2)));
    const i32x4_t rs_sc = buf_rsrc(a.sC, Q8 ? (unsigned)(BLKC ? (size_t)a.sc_rows * (a.ldc >> 7) * 4
                                                                : (size_t)a.M * (a.ldc >> 5))
                                            : 0u);
    // the bias slice of run r (16 features) from LDS: inline asm with its own wait (a plain LDS
    // read would make hipcc drain vmcnt(0): it cannot tell colv from the DMA stages)
    f32x4 bv[4];
    auto load_bias = [&](int nb) {
        const unsigned ba = (unsigned)(size_t)(LDS_AS const float*)(colv + nb);
        asm volatile(
            "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
            "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
            : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
            : "v"(ba)
            : "memory");
    };
    auto epilogue = [&](int pm0, int pn0) {
        int le;  // lane-derived addresses from an opaque copy of the lane id (no hoisting / spills)
        asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
        const int eh = le >> 5, er = le & 31;
#pragma unroll
        for (int run = 0; run < 2; ++run) {
            const int n = pn0 + wc * 64 + 32 * run + 16 * eh;  // the lane's first feature of this run
            load_bias(n);
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) {
                const int m = pm0 + GRP * 128 + mb * 32 + er;
                // run r = acc[fb][mb] elements 4 r .. 4 r + 3 and 8 + 4 r .. (fb = 0 then 1)
                float v[16];
#pragma unroll
                for (int fb = 0; fb < 2; ++fb)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        v[8 * fb + j] = acc[fb][mb][4 * run + j] + bv[2 * fb][j];
                        v[8 * fb + 4 + j] = acc[fb][mb][8 + 4 * run + j] + bv[2 * fb + 1][j];
                    }
                if constexpr (GELU) {
#pragma unroll
                    for (int q = 0; q < 16; q += 2) quick_gelu2(v[q], v[q + 1]);
                }
                if constexpr (Q8) {
                    float am = 0.f;
#pragma unroll
                    for (int q = 0; q < 16; ++q) am = fmaxf(am, fabsf(v[q]));
                    am = fmaxf(am, __shfl_xor(am, 32, 64));  // the block's other 16 features: lane ^ 32
                    const int e = mx_exp(am);
                    const float inv = mx_inv(e);
                    const u32x4 q8 = {pk4_e4m3(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv),
                                      pk4_e4m3(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv),
                                      pk4_e4m3(v[8] * inv, v[9] * inv, v[10] * inv, v[11] * inv),
                                      pk4_e4m3(v[12] * inv, v[13] * inv, v[14] * inv, v[15] * inv)};
                    unsigned co, so;
                    if constexpr (BLKC) {
                        co = m < mpad ? (unsigned)blk8_off(m, n, a.ldc) : 0xFFFFFFF0u;
                        so = m < mpad ? ((unsigned)(n >> 7) * (unsigned)a.sc_rows + (unsigned)m) * 4u + (unsigned)((n >> 5) & 3)
                                      : 0xFFFFFFF0u;
                    } else {
                        co = m < a.M ? (unsigned)m * (unsigned)a.ldc + (unsigned)n : 0xFFFFFFF0u;
                        so = m < a.M ? (unsigned)m * (unsigned)(a.ldc >> 5) + (unsigned)(n >> 5) : 0xFFFFFFF0u;
                    }
                    raw_buffer_store_v4i32(__builtin_bit_cast(i32x4_t, q8), rs_out, (int)co, 0, MX_AUX_ST);
                    // lanes l and l ^ 32 hold the same block scale: both store it (same byte)
                    raw_buffer_store_i8((char)(e + 127), rs_sc, (int)so, 0, 0);
                } else if constexpr (F32) {
                    const unsigned off = m < a.M ? ((unsigned)m * (unsigned)a.ldc + (unsigned)n) * 4u : 0xFFFFFFC0u;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        raw_buffer_store_v4i32(__builtin_bit_cast(i32x4_t, f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]}),
                                               rs_out, (int)(off + 16u * i), 0, MX_AUX_ST16);
                } else {
                    const u32x4 w0 = {pack2<TO>(v[0], v[1]), pack2<TO>(v[2], v[3]), pack2<TO>(v[4], v[5]), pack2<TO>(v[6], v[7])};
                    const u32x4 w1 = {pack2<TO>(v[8], v[9]), pack2<TO>(v[10], v[11]), pack2<TO>(v[12], v[13]), pack2<TO>(v[14], v[15])};
                    const unsigned off = m < a.M ? ((unsigned)m * (unsigned)a.ldc + (unsigned)n) * 2u : 0xFFFFFFE0u;
                    raw_buffer_store_v4i32(__builtin_bit_cast(i32x4_t, w0), rs_out, (int)off, 0, MX_AUX_ST16);
                    raw_buffer_store_v4i32(__builtin_bit_cast(i32x4_t, w1), rs_out, (int)(off + 16u), 0, MX_AUX_ST16);
                }
                __builtin_amdgcn_sched_barrier(0);  // one block at a time (register pressure)
            }
        }
    };
    const i32x4_t rs_drop = buf_rsrc(a.C, 0u);
    auto null_stores = [&]() {  // the first tile: NSTORE dropped stores in the epilogue's place
        const i32x4_t z = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < NSTORE; ++i) raw_buffer_store_v4i32(z, rs_drop, 0, 0, 0);
    };

    // one k-step, compile-time position (as gemm_p32.h's kstep)
    auto kstep = [&](int kk_issue, auto nxt, auto stc, auto stic, auto first, auto ep, auto w24,
                     bool have_prev, int pm0, int pn0) {
        constexpr bool NXT = decltype(nxt)::value;
        constexpr bool EP = decltype(ep)::value;
        constexpr bool W24 = decltype(w24)::value;
        if constexpr (NXT) stage_pieces(rs_n, ss_n, sv_n, kk_issue, decltype(stic)::value);
        else stage_pieces(rs_c, ss_all, sv_c, kk_issue, decltype(stic)::value);
        if constexpr (GRP == 1) {
            if (W24) vm_wait<W_HI>(); else vm_wait<W_LO>();
        }
        if constexpr (EP) {
            if (have_prev) epilogue(pm0, pn0);
            else null_stores();
        }
        reads(stc);
        if constexpr (GRP == 1) __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): WAR of the stage
        bar();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // the fragment reads (inline asm) landed
        __builtin_amdgcn_sched_barrier(0);
        mfmas(first, stc);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (GRP == 0) {
            if (W24) vm_wait<W_HI>(); else vm_wait<W_LO>();
        }
        bar();
    };
    // prologue: steps 0, 1, 2 of the first tile; the bias vector of the whole GEMM -> LDS
    stage_pieces(rs_c, ss_all, sv_c, 0, 0);
    stage_pieces(rs_c, ss_all, sv_c, 1, 1);
    stage_pieces(rs_c, ss_all, sv_c, 2, 2);
    {
        float* cv = (float*)(smem + 4 * STAGE);
        for (int i = (GRP * 256 + wc * 64 + lane); i < a.N; i += 512) cv[i] = a.bias ? a.bias[i] : 0.f;
    }
    vm_wait<0>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if constexpr (GRP == 1) __builtin_amdgcn_s_barrier();  // the stagger

    using T_ = std::true_type;
    using F_ = std::false_type;
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    using S2 = std::integral_constant<int, 2>;
    using S3 = std::integral_constant<int, 3>;
    using W0 = std::integral_constant<bool, GRP == 0>;
    int pm0 = 0, pn0 = 0;
    for (int i = 1;; ++i) {
        const bool have_prev = i > 1;
        kstep(3, F_{}, S0{}, S3{}, T_{}, T_{}, W0{}, have_prev, pm0, pn0);
        kstep(4, F_{}, S1{}, S0{}, F_{}, F_{}, T_{}, false, 0, 0);
        kstep(5, F_{}, S2{}, S1{}, F_{}, F_{}, T_{}, false, 0, 0);
        kstep(6, F_{}, S3{}, S2{}, F_{}, F_{}, F_{}, false, 0, 0);
        for (int kt = 4; kt < nk - 4; kt += 4) {
            kstep(kt + 3, F_{}, S0{}, S3{}, F_{}, F_{}, F_{}, false, 0, 0);
            kstep(kt + 4, F_{}, S1{}, S0{}, F_{}, F_{}, F_{}, false, 0, 0);
            kstep(kt + 5, F_{}, S2{}, S1{}, F_{}, F_{}, F_{}, false, 0, 0);
            kstep(kt + 6, F_{}, S3{}, S2{}, F_{}, F_{}, F_{}, false, 0, 0);
        }
        kstep(nk - 1, F_{}, S0{}, S3{}, F_{}, F_{}, F_{}, false, 0, 0);
        kstep(0, T_{}, S1{}, S0{}, F_{}, F_{}, F_{}, false, 0, 0);
        kstep(1, T_{}, S2{}, S1{}, F_{}, F_{}, F_{}, false, 0, 0);
        kstep(2, T_{}, S3{}, S2{}, F_{}, F_{}, F_{}, false, 0, 0);
        pm0 = m0;
        pn0 = n0;
        if (!has_next) break;
        m0 = mn;
        n0 = nn;
        rs_c = rs_n;
        sv_c = sv_n;
        has_next = tile(i + 1, mn, nn);
        rs_n = has_next ? rsrc_of(mn, nn) : rs_none;
        ss_n = has_next ? ss_all : ss_none;
        sv_n = has_next ? sv_of(mn, nn) : 0u;
    }
    epilogue(pm0, pn0);
    if constexpr (GRP == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
    vm_wait<0>();
}

// LDS: four stages of (256 + 256) x 64 B operands + 2 KB of scale dwords, then the bias vector
// (fp32, N <= 4096): 152 KB
template <typename TO, int EPI, bool BLKC>
__global__ __launch_bounds__(512, 1) void gemm_mx8_p32_kernel(GemmArgs a, int ntiles) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[4 * ((256 + 256) * 64 + (256 + 256) * 4) + 4096 * 4];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave < 4) p32mx_body<TO, EPI, BLKC, 0>(a, ntiles, smem, lane, wave);
    else p32mx_body<TO, EPI, BLKC, 1>(a, ntiles, smem, lane, wave - 4);
}

}  // namespace clipvit
