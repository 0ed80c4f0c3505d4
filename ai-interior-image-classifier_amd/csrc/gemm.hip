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
                for (int i = 0; i < 16; ++i) v[i] *= __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v[i]));
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

// ABL (timing-only ablation builds, results wrong): bit0 no global->LDS loads, bit1 no LDS
// fragment reads, bit2 no MFMAs.
// PRIO: s_setprio(1) around each MFMA cluster (the arbiter then issues a wave's MFMAs ahead of
// the other wave's LDS / global instructions on the same SIMD).
template <typename T, int BM, int BN, int WM, int WN, int NS, int EPI, int SM = 0, int ABL = 0, int PRIO = 0>
__global__ __launch_bounds__(64 * WM* WN) void gemm_pipe_kernel(GemmArgs a) {
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
    __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STAGE];

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
#pragma unroll
    for (int r = 0; r < LA; ++r) {
        const int p = r * NT * 16 + tid * 16;
        const int row = p >> 7, c = ((p >> 4) & 7) ^ (row & 7);
        asrc[r] = (size_t)min(m0 + row, mlast) * ldb + c * 16;
    }
#pragma unroll
    for (int r = 0; r < LW; ++r) {
        const int p = r * NT * 16 + tid * 16;
        const int row = p >> 7, c = ((p >> 4) & 7) ^ (row & 7);
        wsrc[r] = (size_t)(n0 + row) * ldb + c * 16;
    }
    auto stage = [&](int buf, int kt) {
        if constexpr (ABL & 1) return;
        unsigned char* sA = smem + buf * STAGE;
        unsigned char* sW = sA + A_BYTES;
        const size_t kofs = (size_t)kt * 128;
#pragma unroll
        for (int r = 0; r < LA; ++r)
            if (r * NT * 16 + wave * 1024 < A_BYTES)  // wave-uniform
                glds16(Ab + asrc[r] + kofs, sA + r * NT * 16 + wave * 1024);
#pragma unroll
        for (int r = 0; r < LW; ++r)
            if (r * NT * 16 + wave * 1024 < W_BYTES)
                glds16(Wb + wsrc[r] + kofs, sW + r * NT * 16 + wave * 1024);
    };

    const int lrow = lane & 15, lsw = lane & 7, lg = lane >> 4;
    const int aoff = (wm * TM + lrow) * 128, woff = A_BYTES + (wn * TN + lrow) * 128;
    auto load_frags = [&](int buf, int s, vec8 (&af)[FM], vec8 (&wf)[FN]) {
        if constexpr (ABL & 2) {
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) asm volatile("" : "=v"(af[fm]));
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) asm volatile("" : "=v"(wf[fn]));
            return;
        }
        const unsigned char* base = smem + buf * STAGE;
        const int c = (((s << 2) | lg) ^ lsw) << 4;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) af[fm] = *(const vec8*)(base + aoff + fm * 2048 + c);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) wf[fn] = *(const vec8*)(base + woff + fn * 2048 + c);
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Ring protocol: tile t lives in stage t % NS. Prologue issues tiles 0..NS-2; the stage of
    // tile t-1 is refilled with tile t-1+NS right after the barrier that follows every wave's
    // last ds_read of tile t-1 (lgkmcnt(0) before that barrier).
    const int nk = a.K >> 6;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) stage(s, s);
    wait_tile<LPT, NS>(min(NS - 2, nk - 1));
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
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
        if constexpr (ABL & 4) {
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) asm volatile("" ::"v"(af[fm]));
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) asm volatile("" ::"v"(wf[fn]));
        } else {
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
#pragma unroll
                for (int fm = 0; fm < FM; ++fm) acc[fn][fm] = T::mfma16(wf[fn], af[fm], acc[fn][fm]);
        }
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
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
    {   // last tile
        __builtin_amdgcn_s_waitcnt(0xC07F);
        load_frags((nk - 1) % NS, 1, a1, w1);
        mfmas(a0, w0);
        interleave();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        mfmas(a1, w1);
    }

    // ---- epilogue (same contract as gemm_nt_kernel) ----
    const int g = lg;
    if constexpr (SM == 3 && (EPI == EPI_STORE || EPI == EPI_GELU)) {
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
#pragma unroll
            for (int q = 0; q < FN / 4; ++q) {
                const int nl = wn * TN + q * 64 + 16 * g;
                float v[16];
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) v[4 * f + rr] = acc[4 * q + f][fm][rr];
                if (a.bias) {
                    const float4* b4 = (const float4*)(a.bias + n0 + nl);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float4 bb = b4[i];
                        v[4 * i] += bb.x; v[4 * i + 1] += bb.y; v[4 * i + 2] += bb.z; v[4 * i + 3] += bb.w;
                    }
                }
                if constexpr (EPI == EPI_GELU) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) v[i] *= __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v[i]));
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
#pragma unroll 4
        for (int i = tid; i < BM * CPR; i += NT) {
            const int r = i / CPR, c = i % CPR;
            const int m = m0 + r;
            const uint4 val = *(const uint4*)(smem + r * ROWB + ((c ^ (r & 7)) << 4));
            if (m < a.M) *(uint4*)(Cb + ((size_t)m * a.ldc + n0) * 2 + c * 16) = val;
        }
        return;
    }
    OutStore<SM> out(a.C);
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
                for (int i = 0; i < 16; ++i) v[i] *= __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v[i]));
            }
            if constexpr (EPI == EPI_STORE || EPI == EPI_GELU) {
                const size_t off = ((size_t)m * a.ldc + n) * 2;
                out.u4(off, make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]),
                                       pack2<T>(v[6], v[7])));
                out.u4(off + 16, make_uint4(pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]),
                                            pack2<T>(v[12], v[13]), pack2<T>(v[14], v[15])));
            } else if constexpr (EPI == EPI_RESID) {
                const float4* src = (const float4*)((float*)a.C + (size_t)m * a.ldc + n);
                const size_t off = ((size_t)m * a.ldc + n) * 4;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    float4 o = src[i];
                    o.x += v[4 * i]; o.y += v[4 * i + 1]; o.z += v[4 * i + 2]; o.w += v[4 * i + 3];
                    out.f4(off + 16 * i, o);
                }
            } else if constexpr (EPI == EPI_DISCARD) {
                float t = 0.f;
#pragma unroll
                for (int i = 0; i < 16; ++i) t += v[i];
                if (t == 1.2345e-30f) ((float*)a.C)[0] = t;  // never taken; keeps the MFMAs live
            } else {
                size_t row = (size_t)m;
                if constexpr (EPI == EPI_PATCH)
                    row = (size_t)(m / a.patch_g2) * a.patch_ntok + 1 + (m % a.patch_g2);
                const size_t off = (row * a.ldc + n) * 4;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    out.f4(off + 16 * i, make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]));
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Ping-pong GEMM (the production kernel): 256x256 block tile, BK = 32, 8 waves in two groups
// of 4 that run one barrier apart. Group g owns token rows [128 g, 128 g + 128); wave p of a
// group owns features [64 p, 64 p + 64) -> 8 x 4 accumulator tiles of 16x16 per wave.
// Every barrier interval, on every SIMD, one wave issues a 16-MFMA cluster while its partner
// (the other group) reads its next fragments from LDS and issues its share of the
// global->LDS loads, so the matrix pipe never waits on LDS or on a barrier of its own group.
//   per tile, group g:  R0 | M0 | R1 | M1      (R = read phase, M = 16-MFMA cluster)
//   group 1 starts one interval late (one extra s_barrier first; group 0 one extra last).
// LDS: 4-stage ring of 32 KB (A 256 x 32 + W 256 x 32, 16-bit); tile t+3 is loaded while tile t
// is consumed (group 0 loads A rows, group 1 loads W rows, half a tile per read phase), so
// every global load has ~9 intervals to land. Rows are 64 B: 16-B chunk c of row r is stored at
// c ^ ((r >> 2) & 2), which makes each ds_read_b128 fragment read conflict-free; glds writes
// lane-linearly, so the same permutation is applied to the per-lane SOURCE address.
constexpr int PP_BM = 256, PP_BN = 256, PP_NS = 4, PP_STAGE = 32768;

__device__ __forceinline__ void sbar() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// ABL (timing-only ablation builds, results wrong): bit0 no global->LDS loads in the loop,
// bit1 no LDS fragment reads in the loop, bit2 no barriers in the loop, bit3 no MFMAs.
template <typename T, int EPI, int ABL = 0>
__global__ __launch_bounds__(512) void gemm_pp_kernel(GemmArgs a) {
    typedef typename T::vec8 vec8;
    __shared__ __attribute__((aligned(16))) unsigned char smem[PP_NS * PP_STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = wave >> 2, p = wave & 3;
    const int nN = a.N / PP_BN;
    const int nwg = gridDim.x;
    int bid = blockIdx.x;
    {
        const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    }
    const int m0 = (bid / nN) * PP_BM, n0 = (bid % nN) * PP_BN;
    const size_t ldb = (size_t)a.K * 2;
    const int nk = a.K >> 5;

    // ---- global->LDS assignment: group 0 loads A (rows m0..), group 1 loads W (rows n0..);
    // read phase r loads rows [128 r, 128 r + 128) of that operand, 2 x 16 B per thread.
    const unsigned char* src_base = (const unsigned char*)(g == 0 ? a.A : a.W);
    const int tg = tid & 255;
    size_t srcoff[2][2];
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int row = r * 128 + j * 64 + (tg >> 2);
            const int c = (tg & 3) ^ ((row >> 2) & 2);
            const int grow = g == 0 ? min(m0 + row, a.M - 1) : n0 + row;
            srcoff[r][j] = (size_t)grow * ldb + c * 16;
        }
    const int ldsw = g * 16384 + (wave & 3) * 1024;  // wave-uniform part of the glds target
    auto issue = [&](int r, int t) {  // half-tile r of K-tile t into its ring stage
        unsigned char* dst = smem + (t % PP_NS) * PP_STAGE + ldsw + r * 8192;
        const size_t kofs = (size_t)t * 64;
        glds16(src_base + srcoff[r][0] + kofs, dst);
        glds16(src_base + srcoff[r][1] + kofs, dst + 4096);
    };

    // ---- fragment addressing (see swizzle note above)
    const int cs = (((lane >> 4) ^ ((lane >> 2) & 2)) << 4);
    const int arow = (g * 128 + (lane & 15)) * 64 + cs;
    const int wrow = 16384 + (p * 64 + (lane & 15)) * 64 + cs;

    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    vec8 af[4], wf[4];

    // ---- prologue: tiles 0..2 in flight, wait for tile 0 (own loads), publish
#pragma unroll
    for (int t = 0; t < 3; ++t)
        if (t < nk) { issue(0, t); issue(1, t); }
    if (nk >= 3) vm_wait<8>();
    else if (nk == 2) vm_wait<4>();
    else vm_wait<0>();
    sbar();
    if (g == 1 && !(ABL & 4)) sbar();  // stagger: group 1 runs one interval behind

    for (int t = 0; t < nk; ++t) {
        const unsigned char* st = smem + (t % PP_NS) * PP_STAGE;
        const bool more = (ABL & 1) ? false : t + 3 < nk;
        // R0: fragments for cluster 0 (A rows 0-63 of the group, all W), first half-load of t+3
        if (!(ABL & 2) || t == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = *(const vec8*)(st + arow + i * 1024);
#pragma unroll
            for (int i = 0; i < 4; ++i) wf[i] = *(const vec8*)(st + wrow + i * 1024);
        }
        if (more) issue(0, t + 3);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (!(ABL & 4)) sbar();
        // M0
        __builtin_amdgcn_s_setprio(1);
        if constexpr (ABL & 8) {
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[i]), "v"(wf[i]));
        } else {
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < 4; ++fn) acc[fn][fm] = T::mfma16(wf[fn], af[fm], acc[fn][fm]);
        }
        __builtin_amdgcn_s_setprio(0);
        if (!(ABL & 4)) sbar();
        // R1: fragments for cluster 1 (A rows 64-127), second half-load of t+3, tile t+1 landed
        if (!(ABL & 2)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = *(const vec8*)(st + arow + (4 + i) * 1024);
        }
        if (more) issue(1, t + 3);
        {
            const int after = min(2, nk - 2 - t);  // tiles issued after t+1 (4 loads each)
            if (after >= 2) vm_wait<8>();
            else if (after == 1) vm_wait<4>();
            else vm_wait<0>();
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (!(ABL & 4)) sbar();
        // M1
        __builtin_amdgcn_s_setprio(1);
        if constexpr (ABL & 8) {
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[i]), "v"(wf[i]));
        } else {
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < 4; ++fn)
                    acc[fn][4 + fm] = T::mfma16(wf[fn], af[fm], acc[fn][4 + fm]);
        }
        __builtin_amdgcn_s_setprio(0);
        if (!(ABL & 4)) sbar();
    }
    if (g == 0 && !(ABL & 4)) sbar();  // balance the stagger barrier

    // ---- epilogue: lane owns token m and features n .. n+15 of each 64-feature group
    const int lg = lane >> 4, lrow = lane & 15;
#pragma unroll
    for (int fm = 0; fm < 8; ++fm) {
        const int m = m0 + g * 128 + fm * 16 + lrow;
        if (m >= a.M) continue;
        const int n = n0 + p * 64 + 16 * lg;
        float v[16];
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[4 * f + r] = acc[f][fm][r];
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
            for (int i = 0; i < 16; ++i) v[i] *= __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v[i]));
        }
        if constexpr (EPI == EPI_STORE || EPI == EPI_GELU) {
            uint4* dst = (uint4*)((u16*)a.C + (size_t)m * a.ldc + n);
            dst[0] = make_uint4(pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]),
                                pack2<T>(v[6], v[7]));
            dst[1] = make_uint4(pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]), pack2<T>(v[12], v[13]),
                                pack2<T>(v[14], v[15]));
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

template <typename T>
static void launch_pp(hipStream_t s, int epi, const GemmArgs& a) {
    const int nwg = (a.N / PP_BN) * ((a.M + PP_BM - 1) / PP_BM);
    dim3 grid(nwg), block(512);
    switch (epi) {
        case EPI_STORE: gemm_pp_kernel<T, EPI_STORE><<<grid, block, 0, s>>>(a); break;
        case EPI_GELU: gemm_pp_kernel<T, EPI_GELU><<<grid, block, 0, s>>>(a); break;
        case EPI_RESID: gemm_pp_kernel<T, EPI_RESID><<<grid, block, 0, s>>>(a); break;
        case EPI_PATCH: gemm_pp_kernel<T, EPI_PATCH><<<grid, block, 0, s>>>(a); break;
        case EPI_F32: gemm_pp_kernel<T, EPI_F32><<<grid, block, 0, s>>>(a); break;
        case EPI_F32GELU: gemm_pp_kernel<T, EPI_F32GELU><<<grid, block, 0, s>>>(a); break;
    }
}

template <typename T, int BM, int BN, int WM, int WN, int NS, int SM = 0>
static void launch_pipe(hipStream_t s, int epi, const GemmArgs& a) {
    const int nwg = grid_for((a.M + BM - 1) / BM, a.N / BN, a.xcd_n);
    dim3 grid(nwg), block(64 * WM * WN);
    if constexpr (SM != 0) {  // non-temporal / write-through store builds: production epilogues only
        switch (epi) {
            case EPI_STORE: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_STORE, SM><<<grid, block, 0, s>>>(a); break;
            case EPI_GELU: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_GELU, SM><<<grid, block, 0, s>>>(a); break;
            case EPI_RESID: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_RESID, SM><<<grid, block, 0, s>>>(a); break;
            default: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_F32, SM><<<grid, block, 0, s>>>(a); break;
        }
        return;
    }
    switch (epi) {
        case EPI_STORE: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_STORE><<<grid, block, 0, s>>>(a); break;
        case EPI_GELU: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_GELU><<<grid, block, 0, s>>>(a); break;
        case EPI_RESID: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_RESID><<<grid, block, 0, s>>>(a); break;
        case EPI_PATCH: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_PATCH><<<grid, block, 0, s>>>(a); break;
        case EPI_F32: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_F32><<<grid, block, 0, s>>>(a); break;
        case EPI_F32GELU: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_F32GELU><<<grid, block, 0, s>>>(a); break;
        case EPI_DISCARD: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_DISCARD><<<grid, block, 0, s>>>(a); break;
    }
}

template <typename T, int BM, int BN, int WM, int WN, int NS, int SM>
static void launch_pipe_prio(hipStream_t s, int epi, const GemmArgs& a) {
    const int nwg = grid_for((a.M + BM - 1) / BM, a.N / BN, a.xcd_n);
    dim3 grid(nwg), block(64 * WM * WN);
    switch (epi) {
        case EPI_STORE: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_STORE, SM, 0, 1><<<grid, block, 0, s>>>(a); break;
        case EPI_GELU: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_GELU, SM, 0, 1><<<grid, block, 0, s>>>(a); break;
        case EPI_RESID: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_RESID, SM, 0, 1><<<grid, block, 0, s>>>(a); break;
        case EPI_PATCH: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_PATCH, SM, 0, 1><<<grid, block, 0, s>>>(a); break;
        default: gemm_pipe_kernel<T, BM, BN, WM, WN, NS, EPI_F32, SM, 0, 1><<<grid, block, 0, s>>>(a); break;
    }
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

// ---------------------------------------------------------------------------------------
// Fused epilogue for one wave's TM x TN block (shared by the persistent kernel).
template <typename T, int EPI, int FM, int FN>
__device__ __forceinline__ void epilogue_wave(const GemmArgs& a, f32x4 (&acc)[FN][FM], int mbase,
                                              int nbase, int lane) {
    const int g = lane >> 4, lrow = lane & 15;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
        const int m = mbase + fm * 16 + lrow;
        if (m >= a.M) continue;
#pragma unroll
        for (int q = 0; q < FN / 4; ++q) {
            const int n = nbase + q * 64 + 16 * g;
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
                for (int i = 0; i < 16; ++i) v[i] *= __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v[i]));
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
// Persistent pipelined GEMM: grid = min(#tiles, #CUs); block b owns tiles b, b + G, b + 2G, ...
// and runs ONE continuous 2-stage LDS ring over the concatenated k-steps of all its tiles, so
// the first k-tiles of tile i+1 are loaded (and its first fragments read) while tile i's last
// MFMAs and its epilogue run: the per-tile load latency of a 768-deep K is paid once per block.
template <typename T, int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(64 * WM* WN) void gemm_persist_kernel(GemmArgs a) {
    typedef typename T::vec8 vec8;
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    static_assert(TN % 64 == 0 && TM % 16 == 0, "wave tile");
    constexpr int A_BYTES = BM * 128, W_BYTES = BN * 128;
    constexpr int LA = (A_BYTES + NT * 16 - 1) / (NT * 16), LW = (W_BYTES + NT * 16 - 1) / (NT * 16);
    static_assert(A_BYTES % 1024 == 0 && W_BYTES % 1024 == 0, "whole-wave staging pieces");
    constexpr int STAGE = A_BYTES + W_BYTES;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int nN = a.N / BN;
    const int ntiles = nN * ((a.M + BM - 1) / BM);
    const int G = gridDim.x, b = blockIdx.x;
    const int my_tiles = (ntiles - b + G - 1) / G;
    const int nk = a.K >> 6;
    const int S = my_tiles * nk;

    auto tile_origin = [&](int i, int& m0, int& n0) {  // i-th tile of this block
        int t = b + i * G;
        const int q = ntiles >> 3, r = ntiles & 7, x = t & 7;  // bijective XCD remap
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (t >> 3);
        m0 = (t / nN) * BM;
        n0 = (t % nN) * BN;
    };

    const unsigned char* Ab = (const unsigned char*)a.A;
    const unsigned char* Wb = (const unsigned char*)a.W;
    const size_t ldb = (size_t)a.K * 2;
    const int mlast = a.M - 1;
    int arow[LA], acol[LA], wrow[LW], wcol[LW];
#pragma unroll
    for (int r = 0; r < LA; ++r) {
        const int p = r * NT * 16 + tid * 16;
        arow[r] = p >> 7;
        acol[r] = (((p >> 4) & 7) ^ (arow[r] & 7)) * 16;
    }
#pragma unroll
    for (int r = 0; r < LW; ++r) {
        const int p = r * NT * 16 + tid * 16;
        wrow[r] = p >> 7;
        wcol[r] = (((p >> 4) & 7) ^ (wrow[r] & 7)) * 16;
    }
    auto stage = [&](int buf, int step) {
        int m0, n0;
        tile_origin(step / nk, m0, n0);
        const size_t kofs = (size_t)(step % nk) * 128;
        unsigned char* sA = smem + buf * STAGE;
        unsigned char* sW = sA + A_BYTES;
#pragma unroll
        for (int r = 0; r < LA; ++r)
            if (r * NT * 16 + wave * 1024 < A_BYTES)
                glds16(Ab + (size_t)min(m0 + arow[r], mlast) * ldb + kofs + acol[r],
                       sA + r * NT * 16 + wave * 1024);
#pragma unroll
        for (int r = 0; r < LW; ++r)
            if (r * NT * 16 + wave * 1024 < W_BYTES)
                glds16(Wb + (size_t)(n0 + wrow[r]) * ldb + kofs + wcol[r], sW + r * NT * 16 + wave * 1024);
    };

    const int lrow = lane & 15, lsw = lane & 7, lg = lane >> 4;
    const int aoff = (wm * TM + lrow) * 128, woff = A_BYTES + (wn * TN + lrow) * 128;
    auto load_frags = [&](int buf, int s, vec8 (&af)[FM], vec8 (&wf)[FN]) {
        const unsigned char* base = smem + buf * STAGE;
        const int c = (((s << 2) | lg) ^ lsw) << 4;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) af[fm] = *(const vec8*)(base + aoff + fm * 2048 + c);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) wf[fn] = *(const vec8*)(base + woff + fn * 2048 + c);
    };

    f32x4 acc[FN][FM];
    auto zero = [&]() {
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    auto mfmas = [&](const vec8 (&af)[FM], const vec8 (&wf)[FN]) {
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) acc[fn][fm] = T::mfma16(wf[fn], af[fm], acc[fn][fm]);
    };
    auto finish_tile = [&](int step) {
        int m0, n0;
        tile_origin(step / nk, m0, n0);
        epilogue_wave<T, EPI, FM, FN>(a, acc, m0 + wm * TM, n0 + wn * TN, lane);
        zero();
    };

    zero();
    if (S == 0) return;
    stage(0, 0);
    vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (S > 1) stage(1, 1);
    vec8 a0[FM], w0[FN], a1[FM], w1[FN];
    load_frags(0, 0, a0, w0);
    for (int s = 0; s < S - 1; ++s) {
        const int cur = s & 1;
        __builtin_amdgcn_s_waitcnt(0xC07F);
        load_frags(cur, 1, a1, w1);
        mfmas(a0, w0);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // stage `cur` fully read
        vm_wait<0>();                        // step s+1 landed (own loads; also epilogue stores)
        __builtin_amdgcn_s_barrier();
        if (s + 2 < S) stage(cur, s + 2);
        load_frags(cur ^ 1, 0, a0, w0);
        mfmas(a1, w1);
        if ((s + 1) % nk == 0) finish_tile(s);  // next step starts a new tile
    }
    {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        load_frags((S - 1) & 1, 1, a1, w1);
        mfmas(a0, w0);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        mfmas(a1, w1);
        finish_tile(S - 1);
    }
}

// ---------------------------------------------------------------------------------------
// Persistent GEMM with a DEFERRED epilogue (16-bit outputs: EPI_STORE / EPI_GELU).
//
// Why: in a one-tile-per-block GEMM every CU reaches its epilogue at the same moment, so the
// whole output (78.6 MB for c_fc at bs=256) is written in a chip-wide burst while the MFMAs
// idle — measured on MI355X as 25-30 % of c_fc / qkv time (tools/gemm_tune.py --epi 6).
// Here a block owns tiles b, b+G, ... and runs one continuous 2-stage LDS ring over all
// their k-steps (as gemm_persist_kernel). At a tile's end the waves convert their
// accumulators (bias, QuickGELU, 16-bit) into an LDS stash [BM][BN] and go straight on with
// the next tile; the stash is written to HBM during the next tile's first 8 k-steps, one
// fully coalesced 16-B-per-lane global_store per wave per k-step, so the stores overlap MFMAs.
//
// Stash: row pitch BN*2 B, 16-B chunk c of row r at chunk c ^ (r & 7): the epilogue's
// ds_write_b128 (8 rows x one chunk per 8-lane group) and the drain's ds_read_b128 (one row
// per 32 lanes) are both conflict-free. Per k-step (after the barrier): stage(k+2), store of
// the chunk read one step earlier, fragment reads, drain read of the next chunk. vmcnt is
// counted by hand: the glds of step k+1 are waited with the one younger store left in flight.
// Needs nk >= 9 (the 8 drain reads of a stash finish before the next stash is written).
template <typename T, int BM, int BN, int WM, int WN, int EPI, int ABL = 0, bool NTS = false>
__global__ __launch_bounds__(64 * WM* WN) void gemm_defer_kernel(GemmArgs a) {
    // ABL (timing-only ablations, output wrong): bit0 no global stores, bit1 no stash writes
    typedef typename T::vec8 vec8;
    static_assert(EPI == EPI_STORE || EPI == EPI_GELU, "16-bit outputs only");
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    static_assert(TN % 64 == 0 && TM % 16 == 0, "wave tile");
    constexpr int A_BYTES = BM * 128, W_BYTES = BN * 128;
    constexpr int LA = A_BYTES / (NT * 16), LW = W_BYTES / (NT * 16);
    static_assert(LA * NT * 16 == A_BYTES && LW * NT * 16 == W_BYTES, "whole staging rounds");
    constexpr int STAGE = A_BYTES + W_BYTES;
    constexpr int ROWB = BN * 2, CPR = ROWB / 16;     // stash row bytes, 16-B chunks per row
    constexpr int STASH = BM * ROWB;
    constexpr int DRAIN = STASH / (NT * 16);          // drain pieces per thread per tile
    static_assert(DRAIN * NT * 16 == STASH && DRAIN <= 8 && NT % CPR == 0, "drain shape");
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE + STASH];
    unsigned char* const stash = smem + 2 * STAGE;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int nN = a.N / BN, nM = (a.M + BM - 1) / BM;
    const int G = gridDim.x, b = blockIdx.x;
    const int V = grid_for(nM, nN, a.xcd_n);
    int my_tiles = 0;
    for (int mt, nt; b + my_tiles * G < V && tile_of_block(b + my_tiles * G, nM, nN, a.xcd_n, mt, nt);)
        ++my_tiles;
    const int nk = a.K >> 6;
    const int S = my_tiles * nk;
    if (S == 0) return;

    auto tile_origin = [&](int i, int& m0, int& n0) {
        int mt = 0, nt = 0;
        tile_of_block(b + i * G, nM, nN, a.xcd_n, mt, nt);
        m0 = mt * BM;
        n0 = nt * BN;
    };

    const unsigned char* Ab = (const unsigned char*)a.A;
    const unsigned char* Wb = (const unsigned char*)a.W;
    const size_t ldb = (size_t)a.K * 2;
    const int mlast = a.M - 1;
    int arow[LA], acol[LA], wrow[LW], wcol[LW];
#pragma unroll
    for (int r = 0; r < LA; ++r) {
        const int p = r * NT * 16 + tid * 16;
        arow[r] = p >> 7;
        acol[r] = (((p >> 4) & 7) ^ (arow[r] & 7)) * 16;
    }
#pragma unroll
    for (int r = 0; r < LW; ++r) {
        const int p = r * NT * 16 + tid * 16;
        wrow[r] = p >> 7;
        wcol[r] = (((p >> 4) & 7) ^ (wrow[r] & 7)) * 16;
    }
    auto stage = [&](int buf, int step) {
        int m0, n0;
        tile_origin(step / nk, m0, n0);
        const size_t kofs = (size_t)(step % nk) * 128;
        unsigned char* sA = smem + buf * STAGE;
        unsigned char* sW = sA + A_BYTES;
#pragma unroll
        for (int r = 0; r < LA; ++r)
            glds16(Ab + (size_t)min(m0 + arow[r], mlast) * ldb + kofs + acol[r], sA + r * NT * 16 + wave * 1024);
#pragma unroll
        for (int r = 0; r < LW; ++r)
            glds16(Wb + (size_t)(n0 + wrow[r]) * ldb + kofs + wcol[r], sW + r * NT * 16 + wave * 1024);
    };

    const int lrow = lane & 15, lsw = lane & 7, lg = lane >> 4;
    const int aoff = (wm * TM + lrow) * 128, woff = A_BYTES + (wn * TN + lrow) * 128;
    auto load_frags = [&](int buf, int s, vec8 (&af)[FM], vec8 (&wf)[FN]) {
        const unsigned char* base = smem + buf * STAGE;
        const int c = (((s << 2) | lg) ^ lsw) << 4;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) af[fm] = *(const vec8*)(base + aoff + fm * 2048 + c);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) wf[fn] = *(const vec8*)(base + woff + fn * 2048 + c);
    };

    f32x4 acc[FN][FM];
    auto zero = [&]() {
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
    constexpr int NFR = FM + FN, NMF = FM * FN;
    static_assert(NMF >= NFR, "need at least one MFMA per fragment read");
    auto interleave = [&]() {
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NMF - NFR, 0);
    };
    auto mfmas = [&](const vec8 (&af)[FM], const vec8 (&wf)[FN]) {
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) acc[fn][fm] = T::mfma16(wf[fn], af[fm], acc[fn][fm]);
    };

    // accumulators (+bias, QuickGELU) -> 16-bit stash
    // This lane's 16 bias values per 64-column group of the tile, loaded at the tile end. The
    // tile's last k-step issues its DMA only after the stash write, so the vmcnt(0) the
    // compiler puts before the first use of `bq` waits for these loads only.
    float4 bq[FN / 4][4];
    auto bias_load = [&](int n0) {
#pragma unroll
        for (int q = 0; q < FN / 4; ++q)
#pragma unroll
            for (int i = 0; i < 4; ++i) bq[q][i] = ((const float4*)(a.bias + n0 + wn * TN + q * 64 + 16 * lg))[i];
    };
    auto stash_write = [&](int n0) {
        if (ABL & 2) return;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
            const int r = wm * TM + fm * 16 + lrow;
#pragma unroll
            for (int q = 0; q < FN / 4; ++q) {
                const int cl = wn * TN + q * 64 + 16 * lg;  // local column of this lane's 16
                float v[16];
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[4 * f + i] = acc[4 * q + f][fm][i];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    v[4 * i] += bq[q][i].x; v[4 * i + 1] += bq[q][i].y;
                    v[4 * i + 2] += bq[q][i].z; v[4 * i + 3] += bq[q][i].w;
                }
                if constexpr (EPI == EPI_GELU) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) v[i] *= __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * v[i]));
                }
                const int c0 = cl >> 3, x = r & 7;
                // inline asm: a compiler-visible ds_write after an LDS-DMA gets a vmcnt(0)
                // (ordering against the DMA, which never targets the stash); completion is
                // covered by the lgkmcnt(0) before the next barrier
                const u32x4 lo = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
                const u32x4 hi = {pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]), pack2<T>(v[12], v[13]), pack2<T>(v[14], v[15])};
                const unsigned p0 = (unsigned)(uintptr_t)(stash + r * ROWB + ((c0 ^ x) << 4));
                const unsigned p1 = (unsigned)(uintptr_t)(stash + r * ROWB + (((c0 + 1) ^ x) << 4));
                asm volatile("ds_write_b128 %0, %1" : : "v"(p0), "v"(lo) : "memory");
                asm volatile("ds_write_b128 %0, %1" : : "v"(p1), "v"(hi) : "memory");
            }
        }
    };
    int dm0 = 0, dn0 = 0;  // origin of the stashed tile
    auto drain_read = [&](int i) -> uint4 {
        const int L = i * NT + tid, r = L / CPR, c = L % CPR;
        return *(const uint4*)(stash + r * ROWB + ((c ^ (r & 7)) << 4));
    };
    // In-loop drain read as inline asm: a compiler-visible LDS load after an LDS-DMA gets an
    // s_waitcnt vmcnt(0) (the compiler cannot tell the stash from the ring), which would wait
    // for the DMA just issued. The explicit lgkmcnt(0) at the top of the next step (before
    // the store that consumes `d`) covers the read.
    auto drain_read_async = [&](int i, uint4& d) {
        const int L = i * NT + tid, r = L / CPR, c = L % CPR;
        const unsigned addr = (unsigned)(uintptr_t)(stash + r * ROWB + ((c ^ (r & 7)) << 4));
        asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr) : "memory");
    };
    auto drain_store = [&](int i, uint4 d) {
        const int L = i * NT + tid, r = L / CPR, c = L % CPR;
        if (ABL & 1) return;
        if (dm0 + r < a.M) st16<NTS>((u16*)a.C + (size_t)(dm0 + r) * a.ldc + dn0 + c * 8, d);
    };

    zero();
    stage(0, 0);
    vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (S > 1) stage(1, 1);
    vec8 a0[FM], w0[FN], a1[FM], w1[FN];
    load_frags(0, 0, a0, w0);
    int dcnt = DRAIN;      // drain pieces of the stash already read (DRAIN: nothing pending)
    bool dpend = false;    // a piece read last step awaits its store
    bool stored = false;   // a store was issued after the most recent stage()
    uint4 d = make_uint4(0, 0, 0, 0);
    for (int s = 0; s < S - 1; ++s) {
        const int cur = s & 1;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // a0/w0 (and the drain piece) landed
        load_frags(cur, 1, a1, w1);
        mfmas(a0, w0);
        interleave();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // stage `cur` fully read
        if (stored) vm_wait<1>(); else vm_wait<0>();  // step s+1's glds landed
        __builtin_amdgcn_s_barrier();
        const bool tile_end = (s + 1) % nk == 0;
        if (!tile_end && s + 2 < S) stage(cur, s + 2);
        // the previous piece's store is the youngest vm op when the next step waits for this DMA
        stored = dpend;
        if (dpend) drain_store(dcnt - 1, d);
        dpend = dcnt < DRAIN;
        if (dpend) drain_read_async(dcnt++, d);
        load_frags(cur ^ 1, 0, a0, w0);
        mfmas(a1, w1);
        interleave();
        if (tile_end) {  // tile (s / nk) done (nk >= 10: the previous stash is fully drained)
            int tm0, tn0;
            tile_origin(s / nk, tm0, tn0);
            bias_load(tn0);  // this step issued no DMA: the compiler's vmcnt(0) waits for the bias only
            stash_write(tn0);
            dm0 = tm0; dn0 = tn0; dcnt = 0;
            zero();
            if (s + 2 < S) stage(cur, s + 2);
        }
    }
    {   // last step
        __builtin_amdgcn_s_waitcnt(0xC07F);
        load_frags((S - 1) & 1, 1, a1, w1);
        mfmas(a0, w0);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        mfmas(a1, w1);
        __builtin_amdgcn_sched_barrier(0);
        if (dpend) drain_store(dcnt - 1, d);
        int m0, n0;
        tile_origin(my_tiles - 1, m0, n0);
        bias_load(n0);
        stash_write(n0);
        dm0 = m0; dn0 = n0;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    uint4 dl[DRAIN];
#pragma unroll
    for (int i = 0; i < DRAIN; ++i) drain_read_async(i, dl[i]);
    __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
    for (int i = 0; i < DRAIN; ++i) drain_store(i, dl[i]);
}

static int g_num_cus = 0;
static int num_cus() {
    if (!g_num_cus) {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            g_num_cus = n;
        else
            g_num_cus = 256;
    }
    return g_num_cus;
}

template <typename T, int BM, int BN, int WM, int WN>
static void launch_persist(hipStream_t s, int epi, const GemmArgs& a) {
    const int ntiles = (a.N / BN) * ((a.M + BM - 1) / BM);
    const int grid = std::min(ntiles, num_cus());
    dim3 block(64 * WM * WN);
    switch (epi) {
        case EPI_STORE: gemm_persist_kernel<T, BM, BN, WM, WN, EPI_STORE><<<grid, block, 0, s>>>(a); break;
        case EPI_GELU: gemm_persist_kernel<T, BM, BN, WM, WN, EPI_GELU><<<grid, block, 0, s>>>(a); break;
        case EPI_RESID: gemm_persist_kernel<T, BM, BN, WM, WN, EPI_RESID><<<grid, block, 0, s>>>(a); break;
        case EPI_PATCH: gemm_persist_kernel<T, BM, BN, WM, WN, EPI_PATCH><<<grid, block, 0, s>>>(a); break;
        case EPI_F32: gemm_persist_kernel<T, BM, BN, WM, WN, EPI_F32><<<grid, block, 0, s>>>(a); break;
        case EPI_F32GELU: gemm_persist_kernel<T, BM, BN, WM, WN, EPI_F32GELU><<<grid, block, 0, s>>>(a); break;
    }
}

template <typename T, int BM, int BN, int WM, int WN>
static int launch_defer(hipStream_t s, int epi, const GemmArgs& a) {
    if (a.N % BN || a.K < 640 || !a.bias || (epi != EPI_STORE && epi != EPI_GELU)) return -1;
    const int V = grid_for((a.M + BM - 1) / BM, a.N / BN, a.xcd_n);
    const int grid = std::min(V, num_cus());
    dim3 block(64 * WM * WN);
    if (epi == EPI_STORE) gemm_defer_kernel<T, BM, BN, WM, WN, EPI_STORE><<<grid, block, 0, s>>>(a);
    else gemm_defer_kernel<T, BM, BN, WM, WN, EPI_GELU><<<grid, block, 0, s>>>(a);
    return 0;
}

template <typename T, int BM, int BN, int WM, int WN>
static void launch_tile(hipStream_t s, int epi, const GemmArgs& a) {
    const int nwg = (a.N / BN) * ((a.M + BM - 1) / BM);
    dim3 grid(nwg), block(64 * WM * WN);
    switch (epi) {
        case EPI_STORE: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_STORE><<<grid, block, 0, s>>>(a); break;
        case EPI_GELU: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_GELU><<<grid, block, 0, s>>>(a); break;
        case EPI_RESID: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_RESID><<<grid, block, 0, s>>>(a); break;
        case EPI_PATCH: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_PATCH><<<grid, block, 0, s>>>(a); break;
        case EPI_F32: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_F32><<<grid, block, 0, s>>>(a); break;
        case EPI_F32GELU: gemm_nt_kernel<T, BM, BN, WM, WN, EPI_F32GELU><<<grid, block, 0, s>>>(a); break;
    }
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
        case 1:
            if (a.N % 128) return -1;
            launch_tile<T, 128, 128, 2, 2>(s, epi, a);
            return 0;
        case 2:
            if (a.N % 128) return -1;
            launch_tile<T, 256, 128, 4, 2>(s, epi, a);
            return 0;
        case 3:
            if (a.N % 256) return -1;
            launch_tile<T, 256, 256, 2, 4>(s, epi, a);
            return 0;
        case 4:
            if (a.N % 64) return -1;
            launch_tile<T, 64, 64, 4, 1>(s, epi, a);
            return 0;
        case 5:
            if (a.N % 256) return -1;
            launch_tile<T, 128, 256, 2, 4>(s, epi, a);
            return 0;
        case 6:
            if (a.N % 128) return -1;
            launch_tile<T, 256, 128, 2, 2>(s, epi, a);
            return 0;
        case 7:
            if (a.N % 128) return -1;
            launch_tile<T, 128, 128, 4, 2>(s, epi, a);
            return 0;
        // ---- pipelined ring variants ----
        case 8:
            if (a.N % 256) return -1;
            launch_pipe<T, 256, 256, 2, 4, 2>(s, epi, a);
            return 0;
        case 9:
            if (a.N % 256) return -1;
            launch_pipe<T, 128, 256, 2, 4, 3>(s, epi, a);
            return 0;
        case 10:
            if (a.N % 128) return -1;
            launch_pipe<T, 256, 128, 4, 2, 3>(s, epi, a);
            return 0;
        case 11:
            if (a.N % 128) return -1;
            launch_pipe<T, 128, 128, 2, 2, 2>(s, epi, a);
            return 0;
        case 12:
            if (a.N % 128) return -1;
            launch_pipe<T, 128, 128, 2, 2, 4>(s, epi, a);
            return 0;
        case 13:
            if (a.N % 128) return -1;
            launch_pipe<T, 128, 128, 4, 2, 2>(s, epi, a);
            return 0;
        case 14:
            if (a.N % 256) return -1;
            launch_pipe<T, 192, 256, 2, 4, 2>(s, epi, a);
            return 0;
        case 15:
            if (a.N % 256 || a.K % 32) return -1;
            launch_pp<T>(s, epi, a);
            return 0;
        case 21:
            if (a.N % 256) return -1;
            launch_pipe<T, 160, 256, 2, 4, 2>(s, epi, a);
            return 0;
        case 22:
            if (a.N % 128) return -1;
            launch_pipe<T, 160, 128, 2, 2, 2>(s, epi, a);
            return 0;
        case 23:
            if (a.N % 256) return -1;
            launch_pipe<T, 224, 256, 2, 4, 2>(s, epi, a);
            return 0;
        case 28:  // 8 with non-temporal output stores
            if (a.N % 256) return -1;
            launch_pipe<T, 256, 256, 2, 4, 2, 1>(s, epi, a);
            return 0;
        case 29:  // 21 with non-temporal output stores
            if (a.N % 256) return -1;
            launch_pipe<T, 160, 256, 2, 4, 2, 1>(s, epi, a);
            return 0;
        // ---- write-through (sc1) output stores: 50 = 8, 51 = 21, 52 = 13, 53 = 14 ----
        // ---- LDS-staged row-contiguous 16-bit epilogue (SM = 3) of 8 / 13 / 22 ----
        case 80:
            if (a.N % 256) return -1;
            launch_pipe<T, 256, 256, 2, 4, 2, 3>(s, epi, a);
            return 0;
        case 81:
            if (a.N % 128) return -1;
            launch_pipe<T, 128, 128, 4, 2, 2, 3>(s, epi, a);
            return 0;
        case 82:
            if (a.N % 128) return -1;
            launch_pipe<T, 160, 128, 2, 2, 2, 3>(s, epi, a);
            return 0;
        // 224-row tiles: M = 12800 -> 58 M-tiles, i.e. 696 tiles at N = 3072 (2.7 rounds of
        // 256 CUs) with the fill bytes per FLOP of a 256-wide tile
        case 83:
            if (a.N % 256) return -1;
            launch_pipe<T, 224, 256, 2, 4, 2, 3>(s, epi, a);
            return 0;
        case 84:
            if (a.N % 256) return -1;
            launch_pipe<T, 224, 256, 2, 4, 2>(s, epi, a);
            return 0;
        case 85:
            if (a.N % 256) return -1;
            launch_pipe<T, 192, 256, 2, 4, 2, 3>(s, epi, a);
            return 0;
        // 64x64 pipelined tiles with deep rings (the class-token tail's M = B GEMMs: few
        // workgroups, long K, weights cold in cache -> latency-bound; more k-tiles in flight)
        case 90:
            if (a.N % 64) return -1;
            launch_pipe<T, 64, 64, 2, 1, 4>(s, epi, a);
            return 0;
        case 91:
            if (a.N % 64) return -1;
            launch_pipe<T, 64, 64, 2, 1, 8>(s, epi, a);
            return 0;
        // 192-wide tiles for the N = 768 roles (out_proj, c_proj, patch): 4 N-tiles, and with
        // 224 rows 58 x 4 = 232 tiles = ONE round of 256 CUs (160x128: 480 tiles on two
        // workgroups per CU) at 0.0097 B of LDS fill per FLOP instead of 0.0141. 6 waves (2 x 3,
        // 128 x 64 or 112 x 64 per wave), 92 / 94 with the LDS-staged 16-bit epilogue.
        case 92:
            if (a.N % 192) return -1;
            launch_pipe<T, 224, 192, 2, 3, 2, 3>(s, epi, a);
            return 0;
        case 93:
            if (a.N % 192) return -1;
            launch_pipe<T, 224, 192, 2, 3, 2>(s, epi, a);
            return 0;
        case 94:
            if (a.N % 192) return -1;
            launch_pipe<T, 256, 192, 2, 3, 2, 3>(s, epi, a);
            return 0;
        case 95:
            if (a.N % 192) return -1;
            launch_pipe<T, 256, 192, 2, 3, 2>(s, epi, a);
            return 0;
        // 32x64 tiles of ONE wave (class-token tail, M = B rows): twice the workgroups of 64x64
        // and 0.75x the LDS fill bytes per tile, since the tail's long-K GEMMs are bound by
        // the per-CU fill rate on few CUs; 4- / 8-stage ring
        case 96:
            if (a.N % 64) return -1;
            launch_pipe<T, 32, 64, 1, 1, 4>(s, epi, a);
            return 0;
        case 97:
            if (a.N % 64) return -1;
            launch_pipe<T, 32, 64, 1, 1, 8>(s, epi, a);
            return 0;
        // 240x256 tiles for QKV (N = 2304 = 9 x 256): M = 12800 -> 54 M-tiles, 486 tiles =
        // 1.9 rounds of 256 CUs at 0.94x the work per tile, against 450 = 1.76 rounds of
        // 256x256 (whose second round is a full tile time). 98: 12 waves (3 x 4, 80 x 64 per
        // wave: three waves on every SIMD); 99: 6 waves (3 x 2, 80 x 128). LDS-staged epilogue.
        // 256x192 tiles of 12 waves (4 x 3, 64 x 64 per wave: three waves on every SIMD) for
        // the N = 768 roles: 4 N-tiles, 200 tiles at M = 12800 = one round on 200 CUs
        case 89:
            if (a.N % 192) return -1;
            launch_pipe<T, 256, 192, 4, 3, 2, 3>(s, epi, a);
            return 0;
        case 69:  // 89 with direct (unstaged) epilogue stores
            if (a.N % 192) return -1;
            launch_pipe<T, 256, 192, 4, 3, 2>(s, epi, a);
            return 0;
        case 98:
            if (a.N % 256) return -1;
            launch_pipe<T, 240, 256, 3, 4, 2, 3>(s, epi, a);
            return 0;
        case 99:
            if (a.N % 256) return -1;
            launch_pipe<T, 240, 256, 3, 2, 2, 3>(s, epi, a);
            return 0;
        // s_setprio(1) around the MFMA clusters of 80 / 13 / 82
        case 86:
            if (a.N % 256) return -1;
            launch_pipe_prio<T, 256, 256, 2, 4, 2, 3>(s, epi, a);
            return 0;
        case 87:
            if (a.N % 128) return -1;
            launch_pipe_prio<T, 128, 128, 4, 2, 2, 0>(s, epi, a);
            return 0;
        case 88:
            if (a.N % 128) return -1;
            launch_pipe_prio<T, 160, 128, 2, 2, 2, 3>(s, epi, a);
            return 0;
        case 50:
            if (a.N % 256) return -1;
            launch_pipe<T, 256, 256, 2, 4, 2, 2>(s, epi, a);
            return 0;
        case 51:
            if (a.N % 256) return -1;
            launch_pipe<T, 160, 256, 2, 4, 2, 2>(s, epi, a);
            return 0;
        case 52:
            if (a.N % 128) return -1;
            launch_pipe<T, 128, 128, 4, 2, 2, 2>(s, epi, a);
            return 0;
        case 53:
            if (a.N % 256) return -1;
            launch_pipe<T, 192, 256, 2, 4, 2, 2>(s, epi, a);
            return 0;
        // ---- ablations of 8 (timing only, results wrong): 60 no loads, 61 no LDS reads,
        //      62 no MFMAs, 63 MFMAs only (+barriers), 64 loads only (+barriers) ----
        case 60: case 61: case 62: case 63: case 64: {
            if (a.N % 256) return -1;
            const int nwg = grid_for((a.M + 255) / 256, a.N / 256, a.xcd_n);
            const int e = epi == EPI_DISCARD ? EPI_DISCARD : EPI_STORE;
            auto L = [&](auto abl) {
                constexpr int AB = decltype(abl)::value;
                if (e == EPI_DISCARD) gemm_pipe_kernel<T, 256, 256, 2, 4, 2, EPI_DISCARD, 0, AB><<<nwg, 512, 0, s>>>(a);
                else gemm_pipe_kernel<T, 256, 256, 2, 4, 2, EPI_STORE, 0, AB><<<nwg, 512, 0, s>>>(a);
            };
            switch (variant) {
                case 60: L(std::integral_constant<int, 1>{}); break;
                case 61: L(std::integral_constant<int, 2>{}); break;
                case 62: L(std::integral_constant<int, 4>{}); break;
                case 63: L(std::integral_constant<int, 3>{}); break;
                case 64: L(std::integral_constant<int, 6>{}); break;
            }
            return 0;
        }
        // ---- persistent ring variants ----
        case 24:
            if (a.N % 256) return -1;
            launch_persist<T, 160, 256, 2, 4>(s, epi, a);
            return 0;
        case 25:
            if (a.N % 256) return -1;
            launch_persist<T, 256, 256, 2, 4>(s, epi, a);
            return 0;
        case 26:
            if (a.N % 128) return -1;
            launch_persist<T, 128, 128, 4, 2>(s, epi, a);
            return 0;
        case 27:
            if (a.N % 256) return -1;
            launch_persist<T, 128, 256, 2, 4>(s, epi, a);
            return 0;
        // ---- persistent, deferred (LDS-stashed) epilogue; 16-bit outputs only ----
        case 30: return launch_defer<T, 128, 256, 2, 4>(s, epi, a);
        case 31: return launch_defer<T, 128, 256, 4, 2>(s, epi, a);
        case 34: {  // 30 with non-temporal output stores
            if (a.N % 256 || a.K < 640 || !a.bias || (epi != EPI_STORE && epi != EPI_GELU)) return -1;
            const int V = grid_for((a.M + 127) / 128, a.N / 256, a.xcd_n);
            const int grid = std::min(V, num_cus());
            if (epi == EPI_STORE) gemm_defer_kernel<T, 128, 256, 2, 4, EPI_STORE, 0, true><<<grid, 512, 0, s>>>(a);
            else gemm_defer_kernel<T, 128, 256, 2, 4, EPI_GELU, 0, true><<<grid, 512, 0, s>>>(a);
            return 0;
        }
        case 32: case 33: {  // ablations of 30 (timing only): no stores / no stash writes + stores
            if (a.N % 256 || a.K < 640 || !a.bias) return -1;
            const int V = grid_for((a.M + 127) / 128, a.N / 256, a.xcd_n);
            const int grid = std::min(V, num_cus());
            if (variant == 32) gemm_defer_kernel<T, 128, 256, 2, 4, EPI_STORE, 1><<<grid, 512, 0, s>>>(a);
            else gemm_defer_kernel<T, 128, 256, 2, 4, EPI_STORE, 3><<<grid, 512, 0, s>>>(a);
            return 0;
        }
        case 16: case 17: case 18: case 19: case 20: case 65: case 66: {  // ablations (timing only)
            if (a.N % 256 || a.K % 32) return -1;
            const int nwg = (a.N / PP_BN) * ((a.M + PP_BM - 1) / PP_BM);
            const int abl[5] = {1, 2, 4, 3, 7};
            if (variant == 65) { gemm_pp_kernel<T, EPI_F32, 10><<<nwg, 512, 0, s>>>(a); return 0; }  // loads only
            if (variant == 66) { gemm_pp_kernel<T, EPI_F32, 3><<<nwg, 512, 0, s>>>(a); return 0; }   // MFMA only
            switch (abl[variant - 16]) {
                case 1: gemm_pp_kernel<T, EPI_F32, 1><<<nwg, 512, 0, s>>>(a); break;
                case 2: gemm_pp_kernel<T, EPI_F32, 2><<<nwg, 512, 0, s>>>(a); break;
                case 4: gemm_pp_kernel<T, EPI_F32, 4><<<nwg, 512, 0, s>>>(a); break;
                case 3: gemm_pp_kernel<T, EPI_F32, 3><<<nwg, 512, 0, s>>>(a); break;
                case 7: gemm_pp_kernel<T, EPI_F32, 7><<<nwg, 512, 0, s>>>(a); break;
            }
            return 0;
        }
    }
    return -1;
}

int launch_gemm(hipStream_t s, int dtype, int epi, const GemmArgs& a, int variant) {
    if (a.K % 64 != 0 || a.M <= 0) return -1;
    if (variant >= 40 && variant < 50) return launch_gemm_ps(s, dtype, epi, a, variant, num_cus());
    if (variant >= 70 && variant < 80) return launch_gemm_deep(s, dtype, epi, a, variant);
    if (dtype == 2) return launch_t<F16>(s, epi, a, variant);
    return launch_t<BF16>(s, epi, a, variant);
}

}  // namespace clipvit
