// Persistent 256x256 MFMA GEMM with 32-deep k-steps and a four-stage LDS ring (variant 72;
// round 5). Included by gemm_pp.hip, and by tools/probes/gemm_probe.hip with a diagnostic hook
// policy (HK: s_memtime stamps at every barrier and inside the read segment, ablations): one
// source, the library's instantiation (P32NoHooks) compiles every hook to nothing.
//
//   C[M, N] = A[M, K] @ W[N, K]^T + bias   (16-bit C; QuickGELU for c_fc)
//
// What it changes against gemm_ppp_kernel (variant 62), from the r05 timeline probe
// (profiles/r05_gemm_timeline.md): there, a barrier interval of the k-loop took ~490 cycles for
// the 256 cycles of MFMA work in it, and the two wave groups' epilogues ran one after the other
// with no MFMA beside them (~13k of a tile's ~61k cycles). Here:
//  * a k-step is 32 deep and one wave's segment is 32 MFMAs (all 8 x 4 accumulator fragments of
//    its 128 x 64 tile, one k-half), so one barrier interval carries 512 MFMA cycles against
//    12 fragment reads + 4 LDS-DMA pieces of the partner wave (the segment micro-probe:
//    0.95 of the MFMA rate at that ratio);
//  * four 32 KB stages: the k-step t + 3 is staged while t is computed, so every LDS-DMA piece
//    has 4.5-5.5 barrier intervals (~2.5k cycles) to land, against 2-3 in variant 62;
//  * the code of each wave group is a separate compile-time path (group 0 stages A, group 1
//    stages W), and the tile-boundary crossing of the k-step stream is unrolled: the k-loop has
//    no run-time branches; a missing next tile is a zero-length buffer resource (its pieces
//    read as zeros into a stage nobody reads);
//  * the epilogue (bias + QuickGELU for c_fc + conversion + stores) runs in the wave's first read
//    segment of the next tile, after that segment's staging issue; its stores are younger than
//    the staged pieces the next waits count, which allow for them. Its arithmetic is variant
//    62's / the pipelined tiles' (acc from 0, + bias, quick_gelu in common.h), so every tile
//    gives the same bits and the tile choice (per shape, per lane split) never changes a result.
//
// Schedule. Slot = barrier interval. Group g's read segment of k-step t is slot 2t + g, its MFMA
// segment slot 2t + g + 1 (group 1 runs one barrier behind). Stage s = t & 3 is read in slots 2t
// and 2t + 1; group 1 retires its reads (lgkmcnt(0)) before the barrier ending slot 2t + 1, so
// the stage may be refilled from slot 2t + 2: the read segment of step t + 1 stages step t + 4
// (= issue j + 3 in the segment of step j). Every wave waits for ITS pieces of step t + 1 by a
// counted vmcnt before the barrier ending slot 2t + 1 (group 0 after its MFMAs, group 1 after its
// issue), so step t + 1 is complete and visible for both groups' reads.
//
// LDS image of a stage: A rows [256][64 B] then W rows [256][64 B]; 16-B chunk c of row r at
// chunk c ^ ((r >> 2) & 2), which makes the MFMA fragment reads (16 rows x one chunk per
// quarter-wave) conflict-free on ds_read_b128's lane groups; the LDS-DMA writes lane-linearly,
// so the swizzle is in the per-lane global source offset. Blocked A (blk16_off, c_proj's u): a
// 32-deep k-step of a 16-row block is one contiguous 1 KB run, staged verbatim (chunk-major:
// chunk c, row r at c * 256 + r * 16, also conflict-free).
#pragma once
#include <type_traits>

#include "common.h"

// Cache-policy bits of the p32 tile's operand loads (A pieces, W pieces) and epilogue stores
// (gfx950: 1 sc0, 2 nt, 16 sc1; an NT instantiation stores with nt; default stores: GEMM_ST_AUX,
// common.h). Build-time A/B knobs (tools/build_alt.py).
#ifndef P32_AUX_A
#define P32_AUX_A 0
#endif
#ifndef P32_AUX_W
#define P32_AUX_W 0
#endif
#ifndef P32_AUX_ST
#define P32_AUX_ST GEMM_ST_AUX
#endif
#ifndef P32_AUX_NT
#define P32_AUX_NT 2
#endif

namespace clipvit {

// Hook policy of gemm_p32_kernel. The library's: barriers only, no ablation. The probe's policy
// stamps s_memtime in bar() (arrival / departure), at() (points inside a read segment: 0 after
// the staging issue, 1 after group 1's counted wait, 2 after the epilogue, 3 after the fragment
// read issue, 4 after group 1's lgkmcnt(0) drain; in the MFMA segment 5 after its lgkmcnt(0), 6
// after the MFMA issue) and mark() (around the last epilogue).
// ABL (diagnostic builds only; their outputs are garbage): 7 no staging, 8 no MFMA, 9 no
// fragment reads, 3 no epilogue stores.
struct P32NoHooks {
    static constexpr int ABL = 0;
    __device__ __forceinline__ void init(unsigned char*, int, int) {}
    __device__ __forceinline__ void bar(int, int, int) { __builtin_amdgcn_s_barrier(); }
    __device__ __forceinline__ void at(int, int, int) {}
    __device__ __forceinline__ void mark(int, int) {}
    __device__ __forceinline__ void done() {}
};

// NT: non-temporal epilogue stores (variant 74: the large-M c_fc, whose u would otherwise sit
// dirty in the L2 / Infinity Cache in front of the next blocks' operands)
// BM: tile rows, 192, 256 or 320 (variant 79: 192 x 256, each wave 96 x 64; variant 77: 320 x
// 256 tiles, each wave 160 x 64; FM = BM / 32
// accumulator fragments per column slice, NP = the wave's LDS-DMA pieces per k-step: BM / 64
// for group 0 (A), 4 for group 1 (W))
template <typename T, int EPI, bool BLKA, bool BLKW, int GRP, bool NT, int BM, class HK>
__device__ __forceinline__ void p32_body(const GemmArgs& a, int ntiles, unsigned char* smem, int lane, int wc, HK& hk) {
    typedef typename T::vec8 vec8;
    static_assert(BM == 192 || BM == 256 || BM == 320, "p32 tile rows");
    constexpr int BN = 256;
    constexpr int A_ST = BM * 64, STAGE = (BM + BN) * 64;  // 16 / 20 KB + 16 KB
    constexpr int FM = BM / 32, NP = GRP == 0 ? BM / 64 : 4, HALF = BM / 2;
    constexpr bool GELU = EPI == EPI_GELU;
    // this group's staged operand is in the 16-row blocked layout (blk16_off): the blocked A
    // (c_proj's u) or a blocked weight
    constexpr bool OWN_BLK = (GRP == 0 && BLKA) || (GRP == 1 && BLKW);
    const float* const colv = (const float*)(smem + 4 * STAGE);
    const int nM = (a.M + BM - 1) / BM, nN = a.N / BN;
    const int G = gridDim.x;
    const size_t ldb = (size_t)a.K * 2;
    const int nk = a.K >> 5;  // 32-deep k-steps per tile, a multiple of 4

    auto tile = [&](int i, int& m0, int& n0) {
        const int L = blockIdx.x + i * G;
        if (L >= ntiles) return false;
        int mt, nt;
        tile_of_block(L, nM, nN, a.xcd_n, mt, nt);
        m0 = mt * BM;
        n0 = nt * BN;
        return true;
    };
    // this group's operand panel of a tile (A rows for group 0, W rows for group 1)
    const unsigned char* const src = (const unsigned char*)(GRP == 0 ? a.A : a.W);
    const int rows = GRP == 0 ? (BLKA ? (a.M + 15) & ~15 : a.M) : a.N;  // (N % 256 == 0)
    auto rsrc_of = [&](int m0, int n0) {
        const int r0 = GRP == 0 ? m0 : n0;
        const size_t bytes = (size_t)(rows - r0) * ldb;
        return buf_rsrc(src + (size_t)r0 * ldb, (unsigned)(bytes < 0xFFFFFFFFu ? bytes : 0xFFFFFFFFu));
    };
    const i32x4_t rs_none = buf_rsrc(src, 0u);  // no next tile: reads return zeros
    // piece i of this wave = 16 rows 16 p .. 16 p + 15 of the panel, p = NP wc + i
    unsigned voff[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int p = NP * wc + i;
        if constexpr (OWN_BLK) {
            voff[i] = (unsigned)((size_t)p * 16 * ldb + lane * 16);
        } else {
            const int r = lane >> 2, c = (lane & 3) ^ ((lane >> 4) & 2);
            voff[i] = (unsigned)((16 * p + r) * ldb + c * 16);
        }
    }
    const int opbase = GRP == 0 ? 0 : A_ST;
    auto koff = [&](int kk) { return OWN_BLK ? (kk >> 1) * 2048 + (kk & 1) * 1024 : kk * 64; };
    using T_ = std::true_type;
    using F_ = std::false_type;
    auto stage_pieces = [&](const i32x4_t& r, int kk, int st) {
        if constexpr (HK::ABL == 7) return;
        unsigned char* dst = smem + st * STAGE + opbase + NP * wc * 1024;
        const int so = koff(kk);
#pragma unroll
        for (int i = 0; i < NP; ++i) blds16<GRP == 0 ? P32_AUX_A : P32_AUX_W>(r, voff[i], so, dst + i * 1024);
    };

    int m0, n0, mn = 0, nn = 0;
    tile(0, m0, n0);
    bool has_next = tile(1, mn, nn);
    i32x4_t rs_c = rsrc_of(m0, n0), rs_n = has_next ? rsrc_of(mn, nn) : rs_none;

    // fragment addresses: lane (row lrow of a 16-row fragment, k-chunk lg)
    const int lrow = lane & 15, lg = lane >> 4;
    const int swz = ((lg ^ ((lrow >> 2) & 2)) << 4);
    const int aoff = BLKA ? (GRP * HALF / 16) * 1024 + lg * 256 + lrow * 16 : (GRP * HALF + lrow) * 64 + swz;
    constexpr int AFSTEP = BLKA ? 1024 : 1024;  // 16 rows x 64 B either way
    const int woff = BLKW ? A_ST + (wc * 4) * 1024 + lg * 256 + lrow * 16 : A_ST + (wc * 64 + lrow) * 64 + swz;
    vec8 af[FM], wf[4];
    f32x4 acc[4][FM], bv[4];

    // fragment reads by inline asm off two base registers per operand (stages 0 / 1, and 2 / 3
    // 2 STAGE up) with the stage and fragment offsets as immediates below 48 KB. Plain C++ reads
    // made hipcc keep one address register per read (ds_read's offset field is 16 bits and the
    // four stages span 128 KB) and spill. The reads are not visible to hipcc's waitcnt pass: every
    // MFMA segment starts with an explicit lgkmcnt(0) (and a sched_barrier, so nothing that uses
    // a fragment moves above it), and group 1's read segment ends with one.
    unsigned a_lo = (unsigned)(size_t)(LDS_AS unsigned char*)(smem + aoff);
    unsigned w_lo = (unsigned)(size_t)(LDS_AS unsigned char*)(smem + woff);
    unsigned a_hi, w_hi;
    if constexpr (BM == 256) {
        asm volatile("v_add_u32 %0, 0x10000, %2\n\tv_add_u32 %1, 0x10000, %3"
                     : "=v"(a_hi), "=v"(w_hi)
                     : "v"(a_lo), "v"(w_lo));
    } else {
        asm volatile("v_add_u32 %0, %4, %2\n\tv_add_u32 %1, %4, %3"
                     : "=v"(a_hi), "=v"(w_hi)
                     : "v"(a_lo), "v"(w_lo), "s"(2 * STAGE));
    }
    auto rd = [&](vec8& d, unsigned base, auto imm) {
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(base), "i"(decltype(imm)::value));
    };
    auto reads = [&](auto stc) {
        constexpr int ST = decltype(stc)::value, SO = (ST & 1) * STAGE;
        if constexpr (HK::ABL == 9) return;
        const unsigned ba = ST >= 2 ? a_hi : a_lo, bw = ST >= 2 ? w_hi : w_lo;
        rd(wf[0], bw, std::integral_constant<int, SO>{});
        rd(wf[1], bw, std::integral_constant<int, SO + 1024>{});
        rd(wf[2], bw, std::integral_constant<int, SO + 2048>{});
        rd(wf[3], bw, std::integral_constant<int, SO + 3072>{});
        rd(af[0], ba, std::integral_constant<int, SO>{});
        rd(af[1], ba, std::integral_constant<int, SO + 1 * AFSTEP>{});
        rd(af[2], ba, std::integral_constant<int, SO + 2 * AFSTEP>{});
        rd(af[3], ba, std::integral_constant<int, SO + 3 * AFSTEP>{});
        rd(af[4], ba, std::integral_constant<int, SO + 4 * AFSTEP>{});
        rd(af[5], ba, std::integral_constant<int, SO + 5 * AFSTEP>{});
        if constexpr (FM > 6) {
            rd(af[6 % FM], ba, std::integral_constant<int, SO + 6 * AFSTEP>{});
            rd(af[7 % FM], ba, std::integral_constant<int, SO + 7 * AFSTEP>{});
        }
        if constexpr (FM > 8) {
            rd(af[8 % FM], ba, std::integral_constant<int, SO + 8 * AFSTEP>{});
            rd(af[9 % FM], ba, std::integral_constant<int, SO + 9 * AFSTEP>{});
        }
    };
    auto mfmas = [&](auto first) {
        constexpr bool FIRST = decltype(first)::value;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm)
#pragma unroll
            for (int fn = 0; fn < 4; ++fn) {
                if constexpr (HK::ABL == 8) asm volatile("" ::"v"(wf[fn]), "v"(af[fm]));
                else acc[fn][fm] = T::mfma16(wf[fn], af[fm], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[fn][fm]);
            }
        __builtin_amdgcn_s_setprio(0);
    };
    int ti = 0;  // tiles finished by this workgroup (hook policy only)
    auto bar = [&](int step, int seg) {
        __builtin_amdgcn_sched_barrier(0);
        hk.bar(ti, step, seg);
        __builtin_amdgcn_sched_barrier(0);
    };
    // the tile's bias vector slice (16 features per lane) from LDS: inline asm with its own wait
    // (a plain LDS read makes hipcc drain vmcnt(0): it cannot tell colv from the DMA stages)
    auto load_bias = [&](int nb) {
        const unsigned ba = (unsigned)(size_t)(LDS_AS const float*)(colv + nb + wc * 64 + 16 * lg);
        asm volatile(
            "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
            "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
            : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
            : "v"(ba)
            : "memory");
    };
    // C through a range-checked resource: rows >= M (row-major) fall outside it and are dropped,
    // so every epilogue issues exactly 2 FM stores (the counted waits W_HI below rely on it);
    // blocked C keeps the padding rows of its last 16-row block inside the resource (the consumer
    // reads them only into unstored rows). The launcher checks the C bytes fit 32 bits.
    const i32x4_t rs_out = buf_rsrc(a.C, (unsigned)((size_t)(a.blk_c ? ((a.M + 15) & ~15) : a.M) * a.ldc * 2));
    auto epilogue = [&](int pm0, int pn0) {
        // lane-derived addresses recomputed here from an opaque copy of the lane id: hipcc
        // otherwise hoists the per-row offsets of all 16 stores out of the tile loop and spills
        int le;
        asm volatile("v_mov_b32 %0, %1" : "=v"(le) : "v"(lane));
        const int n = pn0 + wc * 64 + 16 * (le >> 4);
        load_bias(pn0);  // the finished tile's bias slice
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
            const int m = pm0 + GRP * HALF + fm * 16 + (le & 15);
            float v[16];
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int rr = 0; rr < 4; rr += 2) {  // v_pk_add_f32
                    const f32x2 s = (f32x2){acc[f][fm][rr], acc[f][fm][rr + 1]} + (f32x2){bv[f][rr], bv[f][rr + 1]};
                    v[4 * f + rr] = s.x;
                    v[4 * f + rr + 1] = s.y;
                }
            if constexpr (GELU) {
#pragma unroll
                for (int q = 0; q < 16; q += 2) quick_gelu2(v[q], v[q + 1]);  // x sigmoid(1.702 x)
            }
            u32x4 w0 = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
            u32x4 w1 = {pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]), pack2<T>(v[12], v[13]), pack2<T>(v[14], v[15])};
            unsigned off, off2;
            if (a.blk_c) {  // blocked C: each quarter-wave already writes 256 contiguous bytes
                off = (unsigned)blk16_off(m, n, a.ldc);
                off2 = off + 256;
            } else {
                // row-major C: lane group g holds features [16g, 16g + 16) of the wave's 64-column
                // slice, so plain stores leave 4 scattered 16-B pieces per row and instruction.
                // One permlane32 swap per dword (groups 2-3 of w0 <-> groups 0-1 of w1) gives
                // w0 = {P0, P1, Q0, Q1} = features [0, 32) and w1 = {P2, P3, Q2, Q3} = [32, 64)
                // (P = first, Q = second half of a group's 16 features): 64 contiguous bytes per
                // row and instruction. Both lanes of a swap pair own the same row (same m).
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const auto r = __builtin_amdgcn_permlane32_swap(w0[d], w1[d], false, false);
                    w0[d] = r[0];
                    w1[d] = r[1];
                }
                const int g = le >> 4;
                off = ((unsigned)m * (unsigned)a.ldc + (unsigned)(n - 16 * g)) * 2u + 32u * (g & 1) + 16u * (g >> 1);
                off2 = off + 64;
            }
            if (m >= a.M && !a.blk_c) off = off2 = 0xFFFFFFF0u;  // outside the resource: dropped
            if constexpr (HK::ABL != 3) {
                raw_buffer_store_v4i32(__builtin_bit_cast(i32x4_t, w0), rs_out, (int)off, 0, NT ? P32_AUX_NT : P32_AUX_ST);
                raw_buffer_store_v4i32(__builtin_bit_cast(i32x4_t, w1), rs_out, (int)off2, 0, NT ? P32_AUX_NT : P32_AUX_ST);
            }
            __builtin_amdgcn_sched_barrier(0);  // one row block at a time (register pressure)
        }
    };

    // vmcnt allowances: W_LO = the two younger issue groups of NP pieces (8 at BM = 256);
    // W_HI (24) when the previous tile's 2 FM epilogue stores are also younger than the awaited
    // pieces. On a workgroup's first tile there is no previous tile: 2 FM stores through a
    // zero-length buffer resource (dropped by the range check) take the epilogue's place, so the
    // counts and the code are the same.
    constexpr int W_LO = 2 * NP, W_HI = 2 * NP + 2 * FM;
    const i32x4_t rs_drop = buf_rsrc(a.C, 0u);
    auto null_stores = [&]() {  // inline asm: hipcc would merge the 2 FM identical stores into one
        const u32x4 z = {0u, 0u, 0u, 0u};
        asm volatile(
            "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
            "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
            "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
            "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
            "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
            "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
            "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0"
            :
            : "v"(z), "s"(rs_drop)
            : "memory");
        if constexpr (FM > 6) {
            asm volatile(
                "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
                "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0"
                :
                : "v"(z), "s"(rs_drop)
                : "memory");
        }
        if constexpr (FM > 8) {
            asm volatile(
                "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0\n\t"
                "buffer_store_dwordx4 %0, off, %1, 0\n\tbuffer_store_dwordx4 %0, off, %1, 0"
                :
                : "v"(z), "s"(rs_drop)
                : "memory");
        }
    };
    //
    // one k-step (compile-time position): ST / STI = stage read / staged; NXT = the staged step
    // belongs to the next tile (kk = step within that tile); FIRST = the tile's first step (its
    // MFMAs start the accumulators from 0; the bias is added in the epilogue); EP = it carries the
    // previous tile's epilogue; W24 =
    // wait allowance W_HI instead of W_LO
    auto kstep = [&](int step, int kk_issue, auto nxt, auto stc, auto stic, auto first, auto ep, auto w24,
                     bool have_prev, int pm0, int pn0) {
        constexpr bool EP = decltype(ep)::value;
        constexpr bool W24 = decltype(w24)::value;
        // ---- read segment: staging issue first (it does not wait for anything), then group 1's
        // counted wait, the previous tile's epilogue (its stores younger than every piece the
        // next waits count), the tile's bias slice, the fragment reads ----
        stage_pieces(decltype(nxt)::value ? rs_n : rs_c, kk_issue, decltype(stic)::value);
        hk.at(ti, step, 0);
        if constexpr (GRP == 1) {  // pieces of step t + 1 (issued two read segments ago) landed
            if (W24) vm_wait<W_HI>(); else vm_wait<W_LO>();
            hk.at(ti, step, 1);
        }
        if constexpr (EP) {
            if (have_prev) epilogue(pm0, pn0);
            else null_stores();
            hk.at(ti, step, 2);
        }
        reads(stc);
        hk.at(ti, step, 3);
        if constexpr (GRP == 1) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): WAR of the stage
            hk.at(ti, step, 4);
        }
        bar(step, 0);
        // ---- MFMA segment ----
        __builtin_amdgcn_s_waitcnt(0xC07F);  // the fragment reads (inline asm) landed
        hk.at(ti, step, 5);
        __builtin_amdgcn_sched_barrier(0);
        mfmas(first);
        __builtin_amdgcn_sched_barrier(0);
        hk.at(ti, step, 6);
        if constexpr (GRP == 0) {
            if (W24) vm_wait<W_HI>(); else vm_wait<W_LO>();
        }
        bar(step, 1);
    };
    // prologue: steps 0, 1, 2 of the first tile; the bias vector of the whole GEMM -> LDS
    stage_pieces(rs_c, 0, 0);
    stage_pieces(rs_c, 1, 1);
    stage_pieces(rs_c, 2, 2);
    {
        float* cv = (float*)(smem + 4 * STAGE);
        for (int i = (GRP * 256 + wc * 64 + lane); i < a.N; i += 512) cv[i] = a.bias ? a.bias[i] : 0.f;
    }
    vm_wait<0>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    if constexpr (GRP == 1) __builtin_amdgcn_s_barrier();  // the stagger

    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    using S2 = std::integral_constant<int, 2>;
    using S3 = std::integral_constant<int, 3>;
    using W0 = std::integral_constant<bool, GRP == 0>;  // group 0 waits after its epilogue's stores
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int m = 0; m < FM; ++m) acc[f][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    int pm0 = 0, pn0 = 0;
    for (int i = 1;; ++i) {
        const bool have_prev = i > 1;
        // first group of four steps (0..3): step 0 carries the previous tile's epilogue
        kstep(0, 3, F_{}, S0{}, S3{}, T_{}, T_{}, W0{}, have_prev, pm0, pn0);
        kstep(1, 4, F_{}, S1{}, S0{}, F_{}, F_{}, T_{}, false, 0, 0);
        kstep(2, 5, F_{}, S2{}, S1{}, F_{}, F_{}, T_{}, false, 0, 0);
        kstep(3, 6, F_{}, S3{}, S2{}, F_{}, F_{}, F_{}, false, 0, 0);
        for (int kt = 4; kt < nk - 4; kt += 4) {
            kstep(kt, kt + 3, F_{}, S0{}, S3{}, F_{}, F_{}, F_{}, false, 0, 0);
            kstep(kt + 1, kt + 4, F_{}, S1{}, S0{}, F_{}, F_{}, F_{}, false, 0, 0);
            kstep(kt + 2, kt + 5, F_{}, S2{}, S1{}, F_{}, F_{}, F_{}, false, 0, 0);
            kstep(kt + 3, kt + 6, F_{}, S3{}, S2{}, F_{}, F_{}, F_{}, false, 0, 0);
        }
        // last group: steps nk - 4 .. nk - 1 stage nk - 1, then the next tile's steps 0, 1, 2
        // (nk >= 8: the launcher refuses K < 256)
        kstep(nk - 4, nk - 1, F_{}, S0{}, S3{}, F_{}, F_{}, F_{}, false, 0, 0);
        kstep(nk - 3, 0, T_{}, S1{}, S0{}, F_{}, F_{}, F_{}, false, 0, 0);
        kstep(nk - 2, 1, T_{}, S2{}, S1{}, F_{}, F_{}, F_{}, false, 0, 0);
        kstep(nk - 1, 2, T_{}, S3{}, S2{}, F_{}, F_{}, F_{}, false, 0, 0);
        pm0 = m0;
        pn0 = n0;
        ++ti;
        if (!has_next) break;
        m0 = mn;
        n0 = nn;
        rs_c = rs_n;
        has_next = tile(i + 1, mn, nn);
        rs_n = has_next ? rsrc_of(mn, nn) : rs_none;
    }
    hk.mark(ti, 0);
    epilogue(pm0, pn0);
    hk.mark(ti, 1);
    if constexpr (GRP == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
    vm_wait<0>();
}

// LDS: four stages of (BM + 256) x 64 B, then the GEMM's bias vector (fp32): 160 KB in all, so
// N <= 8192 at BM = 192 / 256 and N <= 4096 at BM = 320 (launch_p32_t checks)
template <typename T, int EPI, bool BLKA, bool BLKW = false, bool NT = false, int BM = 256, class HK = P32NoHooks>
__global__ __launch_bounds__(512, 1) void gemm_p32_kernel(GemmArgs a, int ntiles) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[4 * 512 * 64 + 8192 * 4];  // 160 KB
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    HK hk;
    hk.init(smem, lane, wave);
    if (wave < 4) p32_body<T, EPI, BLKA, BLKW, 0, NT, BM, HK>(a, ntiles, smem, lane, wave, hk);
    else p32_body<T, EPI, BLKA, BLKW, 1, NT, BM, HK>(a, ntiles, smem, lane, wave - 4, hk);
    hk.done();
}

}  // namespace clipvit
