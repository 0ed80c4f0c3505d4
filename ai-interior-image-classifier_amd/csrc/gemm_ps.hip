// Persistent MFMA GEMM with store-overlapped epilogues (gfx950, wave64).
//
//   C[M, N] = A[M, K] @ W[N, K]^T (+ bias) with the fused epilogues of gemm.hip
//
// Why (measured on MI355X, profiles/r01_gemm_pmc.md): the encoder's K = 768 GEMMs run at
// ~35 % MFMA utilisation at a 2.35 GHz clock, i.e. they are not power-limited but stall on
// (1) the per-tile prologue (two 64 KB LDS stages loaded before the first MFMA) and
// (2) the epilogue (128 KB of fp16 per 256x256 tile written while the MFMAs idle), both paid
// in lock-step by every CU. Here a workgroup owns tiles b, b+G, b+2G, ... (G = #CUs) and runs
// ONE continuous 2-stage LDS ring over the concatenated k-steps of its tiles:
//  * the next tile's first two k-steps are loaded while the current tile finishes, so the
//    prologue is paid once per workgroup, not once per tile;
//  * the epilogue's stores are issued and NOT waited for: the next k-step waits with a counted
//    `s_waitcnt vmcnt(NST)` that leaves exactly the epilogue's NST younger stores in flight;
//  * bias is staged once per launch in LDS (an ordinary global load in the epilogue would make
//    hipcc drain vmcnt to 0, i.e. wait for the next tile's loads and the previous stores).
// Everything else (K-major operands, 16-B XOR-swizzled LDS rows filled by global_load_lds,
// swapped-operand 16x16x32 MFMAs with the packed weight permutation so a lane owns 16
// contiguous output features) is the gemm_pipe_kernel contract.
#include <algorithm>
#include "common.h"

namespace clipvit {

namespace {

constexpr int PS_BIAS_MAX = 5120;  // floats of bias staged in LDS (N <= 4 * 1280)

template <int EPI>
constexpr int stores_per_block() {  // global stores one (fm, 64-feature group) issues
    return (EPI == EPI_STORE || EPI == EPI_GELU) ? 2 : 4;
}

template <typename T, int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(64 * WM* WN) void gemm_ps_kernel(GemmArgs a) {
    typedef typename T::vec8 vec8;
    constexpr int NT = 64 * WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    static_assert(TN % 64 == 0 && TM % 16 == 0, "wave tile");
    constexpr int A_BYTES = BM * 128, W_BYTES = BN * 128;
    static_assert(A_BYTES % (NT * 16) == 0 && W_BYTES % (NT * 16) == 0, "whole staging rounds");
    constexpr int LA = A_BYTES / (NT * 16), LW = W_BYTES / (NT * 16);
    constexpr int STAGE = A_BYTES + W_BYTES;
    constexpr bool HAS_BIAS = EPI != EPI_PATCH;
    constexpr int NST = FM * (FN / 4) * stores_per_block<EPI>();  // stores per lane per tile
    static_assert(NST <= 63, "vmcnt range");
    // one __shared__ object (a second one makes hipcc guard ds_reads with vmcnt(0))
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE + (HAS_BIAS ? PS_BIAS_MAX * 4 : 0)];
    float* sbias = (float*)(smem + 2 * STAGE);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int nN = a.N / BN, nM = (a.M + BM - 1) / BM;
    const int ntiles = nN * nM;
    const int G = gridDim.x, b = blockIdx.x;
    const int my_tiles = b < ntiles ? (ntiles - b + G - 1) / G : 0;
    const int nk = a.K >> 6;
    const int S = my_tiles * nk;

    if constexpr (HAS_BIAS) {  // before any global->LDS load is in flight
        for (int i = tid; i < a.N; i += NT) sbias[i] = a.bias ? a.bias[i] : 0.f;
        __syncthreads();
    }
    if (S == 0) return;

    // i-th tile of this workgroup -> (m0, n0). Workgroups b, b+8, ... share an XCD; the
    // bijective remap gives each such group a contiguous row-major range of logical tiles.
    auto tile_origin = [&](int i, int& m0, int& n0) {
        int t = b + i * G;
        const int q = ntiles >> 3, r = ntiles & 7, x = t & 7;
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
    // acc = bias of the tile's features (so the epilogue needs no bias read). Lane (j, g) of
    // accumulator [fn][*] holds features nbase + 64 (fn / 4) + 16 g + 4 (fn % 4) + r, r < 4.
    // The LDS reads are inline asm: a compiler-visible ds_read of this LDS array is guarded
    // with vmcnt(0) while global->LDS loads are in flight (that would drain the ring).
    auto init_acc = [&](int n0) {
        if constexpr (HAS_BIAS) {
            const unsigned base = (unsigned)(size_t)(const LDS_AS float*)(sbias + n0 + wn * TN + 16 * lg);
            f32x4 bv[FN];
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bv[fn]) : "v"(base), "n"(((fn >> 2) * 64 + (fn & 3) * 4) * 4));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
#pragma unroll
                for (int fm = 0; fm < FM; ++fm) acc[fn][fm] = bv[fn];
        } else {
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
#pragma unroll
                for (int fm = 0; fm < FM; ++fm) acc[fn][fm] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    constexpr int NFR = FM + FN, NMF = FM * FN;
    static_assert(NMF >= NFR, "need at least one MFMA per fragment read");
    auto interleave = [&]() {
#pragma unroll
        for (int i = 0; i < NFR; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NMF - NFR, 0);
    };
    auto mfmas = [&](const vec8 (&af)[FM], const vec8 (&wf)[FN]) {
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) acc[fn][fm] = T::mfma16(wf[fn], af[fm], acc[fn][fm]);
    };

    // Epilogue of the tile at (m0, n0); returns true when every lane issued exactly NST stores.
    auto epilogue = [&](int m0, int n0) -> bool {
        const int mbase = m0 + wm * TM, nbase = n0 + wn * TN;
        const bool full = m0 + BM <= a.M;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
            const int m = mbase + fm * 16 + lrow;
            if (!full && m >= a.M) continue;
#pragma unroll
            for (int q = 0; q < FN / 4; ++q) {
                const int n = nbase + q * 64 + 16 * lg;
                float v[16];
#pragma unroll
                for (int f = 0; f < 4; ++f)
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[4 * f + r] = acc[4 * q + f][fm][r];
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
        // RESID reads C: its loads already waited for everything older, nothing to overlap
        return full && EPI != EPI_RESID;
    };

    {
        int m0, n0;
        tile_origin(0, m0, n0);
        init_acc(n0);
    }
    stage(0, 0);
    if (S > 1) {
        stage(1, 1);
        vm_wait<LA + LW>();  // stage 0 landed, stage 1 may stay in flight
    } else {
        vm_wait<0>();
    }
    __builtin_amdgcn_s_barrier();
    vec8 a0[FM], w0[FN], a1[FM], w1[FN];
    load_frags(0, 0, a0, w0);
    bool stored = false;  // the previous step ended a tile whose NST stores are in flight
    int tile = 0;
    for (int s = 0; s < S; ++s) {
        const int cur = s & 1;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): a0/w0 landed
        load_frags(cur, 1, a1, w1);
        mfmas(a0, w0);
        interleave();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // a1/w1 landed: this wave is done with stage `cur`
        if (s + 1 < S) {
            // stage s+1 was issued one step ago; only the epilogue stores (if any) are younger
            if (stored) vm_wait<NST>();
            else vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();  // every wave done with `cur`; stage s+1 visible to all
        if (s + 2 < S) stage(cur, s + 2);
        if (s + 1 < S) load_frags(cur ^ 1, 0, a0, w0);
        mfmas(a1, w1);
        interleave();
        stored = false;
        if ((s + 1) % nk == 0) {
            int m0, n0;
            tile_origin(tile++, m0, n0);
            stored = epilogue(m0, n0);
            if (tile < my_tiles) {
                tile_origin(tile, m0, n0);
                init_acc(n0);
            }
        }
    }
}

template <typename T, int BM, int BN, int WM, int WN>
int launch_ps_t(hipStream_t s, int epi, const GemmArgs& a, int ncu) {
    if (a.N % BN || a.N > PS_BIAS_MAX) return -1;
    const int ntiles = (a.N / BN) * ((a.M + BM - 1) / BM);
    const int grid = std::min(ntiles, ncu);
    dim3 block(64 * WM * WN);
    switch (epi) {
        case EPI_STORE: gemm_ps_kernel<T, BM, BN, WM, WN, EPI_STORE><<<grid, block, 0, s>>>(a); return 0;
        case EPI_GELU: gemm_ps_kernel<T, BM, BN, WM, WN, EPI_GELU><<<grid, block, 0, s>>>(a); return 0;
        case EPI_RESID: gemm_ps_kernel<T, BM, BN, WM, WN, EPI_RESID><<<grid, block, 0, s>>>(a); return 0;
        case EPI_PATCH: gemm_ps_kernel<T, BM, BN, WM, WN, EPI_PATCH><<<grid, block, 0, s>>>(a); return 0;
        case EPI_F32: gemm_ps_kernel<T, BM, BN, WM, WN, EPI_F32><<<grid, block, 0, s>>>(a); return 0;
        case EPI_F32GELU: gemm_ps_kernel<T, BM, BN, WM, WN, EPI_F32GELU><<<grid, block, 0, s>>>(a); return 0;
    }
    return -1;
}

template <typename T>
int launch_ps_dt(hipStream_t s, int epi, const GemmArgs& a, int variant, int ncu) {
    switch (variant) {
        case 40: return launch_ps_t<T, 256, 256, 2, 4>(s, epi, a, ncu);
        case 41: return launch_ps_t<T, 128, 256, 2, 4>(s, epi, a, ncu);
        case 42: return launch_ps_t<T, 128, 128, 4, 2>(s, epi, a, ncu);
        case 43: return launch_ps_t<T, 256, 128, 4, 2>(s, epi, a, ncu);
    }
    return -1;
}

}  // namespace

// Persistent store-overlapped GEMM variants 40-43 (see launch_gemm in gemm.hip).
int launch_gemm_ps(hipStream_t s, int dtype, int epi, const GemmArgs& a, int variant, int ncu) {
    if (a.K % 64 != 0 || a.M <= 0) return -1;
    if (dtype == 2) return launch_ps_dt<F16>(s, epi, a, variant, ncu);
    return launch_ps_dt<BF16>(s, epi, a, variant, ncu);
}

}  // namespace clipvit
