// GEMM timeline probe (diagnostic build, never shipped):
//   * p32 / p32run: the SHIPPED 32-deep-k-step kernel (csrc/gemm_p32.h, included as is) with the
//     stamp policy P32Stamp (s_memtime at every barrier and at the read / MFMA segments' inner
//     points, in-kernel clock from s_memtime / s_memrealtime) or an ablation policy P32Abl<N>
//     (7 no staging, 8 no MFMA, 9 no fragment reads, 3 no epilogue stores): the per-phase cycle
//     table of profiles/r06_gemm_phases.md, and plain launches for PMC passes;
//   * the persistent ping-pong tile of csrc/gemm_pp.hip (variant 62) as a stamped copy
//     (ppp_probe), with s_memtime at every barrier of the first 12 k-tiles of a workgroup's first
//     three tiles; stamps go to the unused part of the bias area of LDS by inline-asm ds_write
//     (invisible to the waitcnt pass, so the counted vmcnt of the staging pipeline is untouched);
//   * bar: barrier / MFMA-segment micro-probes.
//
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm --amdgpu-mfma-vgpr-form \
//       -o tools/probes/gemm_probe tools/probes/gemm_probe.hip
// ./gemm_probe p32 M N K epi xcd [balanced] | p32run M N K epi xcd iters kind | bar | M N K epi xcd [iters] [grid]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../ai-interior-image-classifier_amd/csrc/common.h"
#include "../../ai-interior-image-classifier_amd/csrc/gemm_p32.h"  // the shipped kernel, with a hook policy below

using namespace clipvit;

constexpr int NST = 512;           // stamps per wave
constexpr int ST_TILES = 3, ST_KT = 12;
constexpr int ST_PER_TILE = 16 * ST_KT + 4;  // depart [8 kt + e], arrive [8 ST_KT + 8 kt + e]

__device__ __forceinline__ void stamp_at(unsigned* sbuf, int lane, int idx) {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    if (lane == 0 && idx < NST) {
        const unsigned a = (unsigned)(size_t)(LDS_AS unsigned*)(sbuf + idx);
        const unsigned v = (unsigned)t;
        asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
    }
}

template <typename T, int EPI, int ABL, bool STAMP>
__global__ __launch_bounds__(512, 1) void ppp_probe(GemmArgs a, int ntiles, unsigned* trace) {
    typedef typename T::vec8 vec8;
    constexpr int BM = 256, BN = 256;
    constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
    constexpr int NBIAS = 8192;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE + NBIAS * 4];  // 160 KB
    float* const colv = (float*)(smem + 2 * STAGE);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wc = wave & 3;
    unsigned* const sbuf = (unsigned*)(colv + 4096) + wave * NST;  // N <= 4096 in the probe
    unsigned long long t_mem0 = 0, t_real0 = 0;
    if constexpr (STAMP) {
        t_mem0 = __builtin_amdgcn_s_memtime();
        t_real0 = __builtin_amdgcn_s_memrealtime();
    }
    const int nM = (a.M + BM - 1) / BM, nN = a.N / BN;
    const int G = gridDim.x;
    const size_t ldb = (size_t)a.K * 2;
    const int nk = a.K >> 6;

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
    const int rows = grp == 0 ? a.M : a.N;
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
        voff[i] = (unsigned)((pc * 8 + lr) * ldb + chunk * 16);
    }
    const int opbase = grp == 0 ? 0 : A_BYTES;

    int m0, n0, mn = 0, nn = 0;
    tile(0, m0, n0);
    bool has_next = tile(1, mn, nn);
    i32x4_t rs_c = rsrc_of(m0, n0), rs_n = has_next ? rsrc_of(mn, nn) : rs_c;
    auto issue = [&](int part, int j) {
        if constexpr (ABL == 7) {
            if (j >= 2) return;
        }
        i32x4_t r = rs_c;
        int kk = j;
        if (j >= nk) {
            if (!has_next) return;
            r = rs_n;
            kk = j - nk;
        }
        unsigned char* dst = smem + (j & 1) * STAGE + opbase;
#pragma unroll
        for (int i = 0; i < 2; ++i) blds16(r, voff[2 * part + i], kk * 128, dst + (8 * part + 2 * wc + i) * 1024);
    };
    f32x4 acc[4][8];
#pragma unroll
    for (int p = 0; p < 4; ++p) issue(p, 0);
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
    if (grp == 1) __builtin_amdgcn_s_barrier();

    const int lrow = lane & 15, lsw = lane & 7, lg = lane >> 4;
    const int woff = A_BYTES + (wc * 64 + lrow) * 128;
    const int c0 = ((0 | lg) ^ lsw) << 4, c1 = ((4 | lg) ^ lsw) << 4;
    const int aoff = (grp * 128 + lrow) * 128;
    vec8 af[4][2], wf[4][2];
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    int ti = 0;  // tiles done by this workgroup (stamp slots)
    // barrier e of k-tile kt; stamped build: s_memtime on arrival (no wait: the wave's reads stay
    // in flight across the barrier as in the plain build) and on departure, then one lgkmcnt(0)
    // (the plain build waits lgkmcnt(0) right after every read-segment barrier anyway)
    auto bar = [&](int kt, int e) {
        if constexpr (STAMP) {
            if (ti < ST_TILES && kt < ST_KT) {
                unsigned long long ta, td;
                asm volatile("s_memtime %0\n\ts_barrier\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)"
                             : "=&s"(ta), "=&s"(td)::"memory");
                if (lane == 0) {
                    const unsigned i0 = 8 + ti * ST_PER_TILE + 8 * kt + e, i1 = i0 + 8 * ST_KT;
                    const unsigned a0 = (unsigned)(size_t)(LDS_AS unsigned*)(sbuf + i0);
                    const unsigned a1 = (unsigned)(size_t)(LDS_AS unsigned*)(sbuf + i1);
                    const unsigned v0 = (unsigned)td, v1 = (unsigned)ta;
                    asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %2, %3" ::"v"(a0), "v"(v0), "v"(a1), "v"(v1) : "memory");
                }
                return;
            }
        }
        __builtin_amdgcn_s_barrier();
    };
#define MFMA_OR_SINK(C, Wf, Af, ZERO)                                      \
    do {                                                                   \
        if constexpr (ABL == 8) asm volatile("" ::"v"(Wf), "v"(Af));      \
        else C = T::mfma16(Wf, Af, (ZERO) ? zero : C);                     \
    } while (0)
    auto ktile = [&](const int kt, const unsigned char* stg, auto Zc) {
        constexpr bool Z = decltype(Zc)::value;
        const bool more = kt + 2 < nk || has_next;
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            wf[f][0] = *(const vec8*)(stg + woff + f * 2048 + c0);
            wf[f][1] = *(const vec8*)(stg + woff + f * 2048 + c1);
        }
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            af[f][0] = *(const vec8*)(stg + aoff + f * 2048 + c0);
            af[f][1] = *(const vec8*)(stg + aoff + f * 2048 + c1);
        }
        if (grp == 0) issue(1, kt + 1); else issue(2, kt + 1);
        __builtin_amdgcn_sched_barrier(0);
        bar(kt, 0);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int fn = 0; fn < 2; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) MFMA_OR_SINK(acc[fn][fm], wf[fn][s], af[fm][s], Z && s == 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        bar(kt, 1);
#pragma unroll
        for (int f = 2; f < 4; ++f) {
            wf[f][0] = *(const vec8*)(stg + woff + f * 2048 + c0);
            wf[f][1] = *(const vec8*)(stg + woff + f * 2048 + c1);
        }
        if (grp == 0) issue(2, kt + 1); else issue(3, kt + 1);
        __builtin_amdgcn_sched_barrier(0);
        bar(kt, 2);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int fn = 2; fn < 4; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) MFMA_OR_SINK(acc[fn][fm], wf[fn][s], af[fm][s], Z && s == 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        bar(kt, 3);
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            af[f][0] = *(const vec8*)(stg + aoff + (f + 4) * 2048 + c0);
            af[f][1] = *(const vec8*)(stg + aoff + (f + 4) * 2048 + c1);
        }
        if (grp == 0) issue(3, kt + 1); else issue(0, kt + 2);
        __builtin_amdgcn_sched_barrier(0);
        bar(kt, 4);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int fn = 2; fn < 4; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) MFMA_OR_SINK(acc[fn][fm + 4], wf[fn][s], af[fm][s], Z && s == 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        bar(kt, 5);
        if (grp == 0) {
            issue(0, kt + 2);
        } else {
            issue(1, kt + 2);
            if (more) vm_wait<4>(); else vm_wait<0>();
        }
        __builtin_amdgcn_sched_barrier(0);
        bar(kt, 6);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int fn = 0; fn < 2; ++fn)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) MFMA_OR_SINK(acc[fn][fm + 4], wf[fn][s], af[fm][s], Z && s == 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (grp == 0) {
            if (more) vm_wait<2>(); else vm_wait<0>();
        }
        bar(kt, 7);
    };
#undef MFMA_OR_SINK
    if constexpr (ABL == 8) {
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int m = 0; m < 8; ++m) acc[f][m] = zero;
    }
    constexpr bool GELU = EPI == EPI_GELU;
    unsigned char* const Cb = (unsigned char*)a.C;
    for (int i = 1;; ++i) {
        ktile(0, smem, std::true_type{});
        ktile(1, smem + STAGE, std::false_type{});
        for (int kt = 2; kt < nk; kt += 2) {
            ktile(kt, smem, std::false_type{});
            ktile(kt + 1, smem + STAGE, std::false_type{});
        }
        if constexpr (STAMP) {
            if (ti < ST_TILES) stamp_at(sbuf, lane, 8 + ti * ST_PER_TILE + 16 * ST_KT + 0);
        }
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
            const bool live = ABL == 3 ? (m < a.M && a.ldc > (1 << 30)) : m < a.M;
            if (live) {
                const size_t off = a.blk_c ? blk16_off(m, n, a.ldc) : ((size_t)m * a.ldc + n) * 2;
                const size_t off2 = a.blk_c ? off + 256 : off + 16;
                const u32x4 w0 = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
                const u32x4 w1 = {pack2<T>(v[8], v[9]), pack2<T>(v[10], v[11]), pack2<T>(v[12], v[13]),
                                  pack2<T>(v[14], v[15])};
                *(u32x4*)(Cb + off) = w0;
                *(u32x4*)(Cb + off2) = w1;
            } else if constexpr (ABL == 3) {
                asm volatile("" ::"v"(v[0]), "v"(v[5]), "v"(v[10]), "v"(v[15]));
            }
        }
        if constexpr (STAMP) {
            if (ti < ST_TILES) stamp_at(sbuf, lane, 8 + ti * ST_PER_TILE + 16 * ST_KT + 1);
        }
        ++ti;
        if (!has_next) break;
        m0 = mn;
        n0 = nn;
        rs_c = rs_n;
        has_next = tile(i + 1, mn, nn);
        if (has_next) rs_n = rsrc_of(mn, nn);
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();
    if constexpr (STAMP) {
        const unsigned long long t_mem1 = __builtin_amdgcn_s_memtime();
        const unsigned long long t_real1 = __builtin_amdgcn_s_memrealtime();
        __syncthreads();
        unsigned* out = trace + ((size_t)blockIdx.x * 8 + wave) * NST;
        for (int i = 8 + lane; i < NST; i += 64) out[i] = sbuf[i];
        if (lane == 0) {
            out[0] = (unsigned)t_mem0;
            out[1] = (unsigned)(t_mem0 >> 32);
            out[2] = (unsigned)t_real0;
            out[3] = (unsigned)(t_real0 >> 32);
            out[4] = (unsigned)t_mem1;
            out[5] = (unsigned)(t_mem1 >> 32);
            out[6] = (unsigned)t_real1;
            out[7] = (unsigned)(t_real1 >> 32);
        }
    }
}


// ---- hook policies for variant 72 (gemm_p32.h's HK parameter) ----
// Stamps: s_memtime (+ lgkmcnt(0), so a stamp never reads a pending SGPR) written by lane 0 into the
// unused part of the bias area of LDS by inline-asm ds_write (invisible to the waitcnt pass: the
// counted vmcnt of the staging pipeline is untouched), copied to g_p32_trace at exit. Per k-step of
// the first two tiles: the four barrier stamps (arrival / departure of the read and MFMA
// segments' closing barriers) and the at() points: 0 after the staging issue, 1 after group 1's
// counted vm wait, 2 after the epilogue, 3 after the fragment reads (group 1 only; the stamp's
// own lgkmcnt(0) drains them, which group 1 does next anyway), 5 after the MFMA segment's
// lgkmcnt(0), 6 after the MFMA issue (group 0's vm wait follows).
constexpr int P32_STEP = 10, P32_TILE = 24 * P32_STEP;
__device__ unsigned* g_p32_trace;
template <int AB = 0>
struct P32Abl {  // ablation only, no stamps
    static constexpr int ABL = AB;
    __device__ __forceinline__ void init(unsigned char*, int, int) {}
    __device__ __forceinline__ void bar(int, int, int) { __builtin_amdgcn_s_barrier(); }
    __device__ __forceinline__ void at(int, int, int) {}
    __device__ __forceinline__ void mark(int, int) {}
    __device__ __forceinline__ void done() {}
};
struct P32Stamp {
    static constexpr int ABL = 0;
    unsigned* sbuf;
    int lane, wave;
    unsigned long long m0, r0;
    __device__ void init(unsigned char* smem, int l, int w) {
        sbuf = (unsigned*)(smem + 4 * 512 * 64) + 4096 + w * NST;  // N <= 4096
        lane = l;
        wave = w;
        m0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    __device__ void put(int idx, unsigned v) {
        if (lane == 0 && idx < NST) {
            const unsigned a = (unsigned)(size_t)(LDS_AS unsigned*)(sbuf + idx);
            asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
        }
    }
    __device__ void bar(int ti, int step, int seg) {
        if (ti < 2 && step < 24) {
            unsigned long long ta, td;
            asm volatile("s_memtime %0\n\ts_barrier\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)" : "=&s"(ta), "=&s"(td)::"memory");
            const int i = 8 + ti * P32_TILE + step * P32_STEP + seg * 2;
            put(i, (unsigned)ta);
            put(i + 1, (unsigned)td);
        } else {
            __builtin_amdgcn_s_barrier();
        }
    }
    __device__ void at(int ti, int step, int pt) {
        if (ti < 2 && step < 24 && pt != 4) {
            unsigned long long t;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
            put(8 + ti * P32_TILE + step * P32_STEP + 4 + (pt > 4 ? pt - 1 : pt), (unsigned)t);
        }
    }
    __device__ void mark(int ti, int which) {
        unsigned long long t;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        put(8 + 2 * P32_TILE + which, (unsigned)t);
    }
    __device__ void done() {
        const unsigned long long m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        __syncthreads();
        unsigned* out = g_p32_trace + ((size_t)blockIdx.x * 8 + wave) * NST;
        for (int i = 8 + lane; i < NST; i += 64) out[i] = sbuf[i];
        if (lane == 0) {
            out[0] = (unsigned)m0; out[1] = (unsigned)(m0 >> 32);
            out[2] = (unsigned)r0; out[3] = (unsigned)(r0 >> 32);
            out[4] = (unsigned)m1; out[5] = (unsigned)(m1 >> 32);
            out[6] = (unsigned)r1; out[7] = (unsigned)(r1 >> 32);
        }
    }
};

// ---- host ----
__global__ void fill_f16(u16* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed * 0x9E3779B9u;
        x ^= x >> 15;
        x *= 0x2c1b3c6dU;
        x ^= x >> 12;
        const float f = ((x >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
        p[i] = __builtin_bit_cast(u16, (_Float16)f);
    }
}
// reference: C[m][n] = sum_k A[m][k] W[p(n)][k] (+ bias, QuickGELU) in fp32; p = the packed row
__global__ void ref_gemm(const u16* A, const u16* W, const float* bias, float* C, int M, int N, int K, int gelu) {
    const int m = blockIdx.y, n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N || m >= M) return;
    const int j = n & 63, i = 4 * (j >> 4) + (j & 3), f = (j & 15) >> 2;
    const int p = (n & ~63) + 16 * f + i;
    float s = 0.f;
    for (int k = 0; k < K; ++k)
        s += (float)__builtin_bit_cast(_Float16, A[(size_t)m * K + k]) * (float)__builtin_bit_cast(_Float16, W[(size_t)p * K + k]);
    s += bias[n];
    if (gelu) s = s / (1.f + expf(-1.702f * s));
    C[(size_t)m * N + n] = s;
}

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)


// ---- barrier / MFMA-segment micro-probe: MFMAs on register operands, no memory ----
// MODE 0: ping-pong (waves >= 4 start one barrier late; per iteration MPS MFMAs, barrier,
// barrier: one wave of each SIMD computes while its partner sits in an empty "read" segment);
// MODE 1: every wave MPS MFMAs then one barrier; MODE 2: no barriers.
template <int WAVES, int MPS, int MODE>
__global__ __launch_bounds__(WAVES * 64, 1) void mfma_bar_probe(float* out, unsigned* cyc, int iters) {
    typedef F16::vec8 vec8;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    vec8 a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (_Float16)(0.001f * (lane + i));
        b[i] = (_Float16)(0.002f * (lane - i));
    }
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 0 && wave >= WAVES / 2) __builtin_amdgcn_s_barrier();
    for (int it = 0; it < iters; ++it) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int m = 0; m < MPS; ++m) acc[m & 15] = F16::mfma16(a, b, acc[m & 15]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (MODE == 0) {
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_s_barrier();
        } else if (MODE == 1) {
            __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (MODE == 0 && wave < WAVES / 2) __builtin_amdgcn_s_barrier();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float sum = 0.f;
    for (int i = 0; i < 16; ++i) sum += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * WAVES * 64 + threadIdx.x] = sum;
    if (lane == 0) cyc[blockIdx.x * WAVES + wave] = (unsigned)(t1 - t0);
}

template <int WAVES, int MPS, int MODE>
static void bar_case(const char* name, int iters) {
    float* out;
    unsigned* cyc;
    CK(hipMalloc(&out, 256 * WAVES * 64 * 4));
    CK(hipMalloc(&cyc, 256 * WAVES * 4));
    for (int r = 0; r < 3; ++r) mfma_bar_probe<WAVES, MPS, MODE><<<256, WAVES * 64>>>(out, cyc, iters);
    CK(hipDeviceSynchronize());
    std::vector<unsigned> c(256 * WAVES);
    CK(hipMemcpy(c.data(), cyc, c.size() * 4, hipMemcpyDeviceToHost));
    std::sort(c.begin(), c.end());
    const double med = c[c.size() / 2];
    // MFMAs per SIMD per iteration: WAVES / 4 waves x MPS
    const double per_it = med / iters, mf = (double)WAVES / 4 * MPS;
    printf("%-34s %7.1f cyc/iter, %5.2f cyc per MFMA per SIMD (ideal 16), MFMA-issue busy %.2f\n", name, per_it,
           per_it / mf, 16.0 * mf / per_it);
    CK(hipFree(out));
    CK(hipFree(cyc));
}


// ---- ping-pong segment probe: what LDS reads and LDS-DMA issue in the partner's segment cost.
// 8 waves, waves 4-7 one barrier late; per iteration every wave runs [read segment: NREAD
// ds_read_b128 + NDMA buffer_load ... lds pieces (L2-resident source), vmcnt keeping two segments
// in flight] barrier [lgkmcnt(0), MPS MFMAs on the fragments just read] barrier.
// SRC: 0 = every workgroup reads the same 1 MB window (L2 hits), 1 KB contiguous per piece;
// 1 = each workgroup streams its own 1 MB (256 MB in all: L2 misses); 2 / 3 = the same with the
// row-major operand pattern of gemm_p32 (16 rows x 64 B per piece, rows 1536 B apart)
template <int MPS, int NDMA, int NREAD, int SRC = 0>
__global__ __launch_bounds__(512, 1) void pp_seg_probe(const unsigned char* src, float* out, unsigned* cyc, int iters) {
    typedef F16::vec8 vec8;
    __shared__ __attribute__((aligned(16))) unsigned char smem[160 * 1024];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = wave >> 2;
    for (int i = threadIdx.x; i < 160 * 1024 / 4; i += 512) ((float*)smem)[i] = 0.001f * (i & 255);
    __syncthreads();
    const i32x4_t rs = buf_rsrc(src + ((SRC & 1) ? (size_t)blockIdx.x * (2u << 20) : 0), 2u << 20);
    const unsigned voff = (SRC & 2) ? (unsigned)((16 * wave + (lane >> 2)) * 1536 + (lane & 3) * 16)
                                    : (unsigned)(wave * 1024 + lane * 16);
    constexpr int NR = NREAD > 0 ? NREAD : 1;
    vec8 fr[NR];
    vec8 b;
    for (int i = 0; i < 8; ++i) b[i] = (_Float16)(0.002f * (lane - i));
    for (int r = 0; r < NR; ++r) fr[r] = b;
    f32x4 acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (grp == 1) __builtin_amdgcn_s_barrier();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < NREAD; ++r)
            fr[r] = *(const vec8*)(smem + 65536 + ((wave * NREAD + r) * 1024 + lane * 16) % 65536);
#pragma unroll
        for (int d = 0; d < NDMA; ++d)
            blds16(rs, voff, (SRC & 2) ? ((it * NDMA + d) & 31) * 64 + (((it * NDMA + d) >> 5) & 3) * 196608
                                       : ((it * NDMA + d) * 8192) & ((1 << 20) - 1),
                   smem + ((d * 8 + wave) * 1024) % 65536);
        if constexpr (NDMA > 0) vm_wait<2 * NDMA>();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < NR; ++r) asm volatile("" ::"v"(fr[r]));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int m = 0; m < MPS; ++m) acc[m & 15] = F16::mfma16(fr[m % NR], b, acc[m & 15]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();
    vm_wait<0>();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float sum = 0.f;
    for (int i = 0; i < 16; ++i) sum += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 512 + threadIdx.x] = sum;
    if (lane == 0) cyc[blockIdx.x * 8 + wave] = (unsigned)(t1 - t0);
}

template <int MPS, int NDMA, int NREAD, int SRC = 0>
static void seg_case(const unsigned char* src, int iters) {
    float* out;
    unsigned* cyc;
    CK(hipMalloc(&out, 256 * 512 * 4));
    CK(hipMalloc(&cyc, 256 * 8 * 4));
    for (int r = 0; r < 3; ++r) pp_seg_probe<MPS, NDMA, NREAD, SRC><<<256, 512>>>(src, out, cyc, iters);
    CK(hipDeviceSynchronize());
    std::vector<unsigned> c(256 * 8);
    CK(hipMemcpy(c.data(), cyc, c.size() * 4, hipMemcpyDeviceToHost));
    std::sort(c.begin(), c.end());
    const double per_int = (double)c[c.size() / 2] / iters / 2;  // two intervals per iteration
    printf("segment: %3d MFMA | partner %2d ds_read_b128 + %d LDS-DMA (src %d): %6.1f cyc per interval (MFMA %d, busy %.2f)\n",
           MPS, NREAD, NDMA, SRC, per_int, MPS * 16, MPS * 16 / per_int);
    CK(hipFree(out));
    CK(hipFree(cyc));
}

template <int EPI, int ABL, bool STAMP>
static void launch(const GemmArgs& a, int grid, int ntiles, unsigned* tr) {
    ppp_probe<F16, EPI, ABL, STAMP><<<grid, 512>>>(a, ntiles, tr);
}
typedef void (*LaunchFn)(const GemmArgs&, int, int, unsigned*);
template <int EPI>
static LaunchFn pick(int abl, bool stamp) {
    if (stamp) return launch<EPI, 0, true>;
    switch (abl) {
        case 3: return launch<EPI, 3, false>;
        case 7: return launch<EPI, 7, false>;
        case 8: return launch<EPI, 8, false>;
        default: return launch<EPI, 0, false>;
    }
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "bar") {
        bar_case<8, 16, 2>("8 waves, no barriers", 2000);
        bar_case<8, 16, 0>("8 waves ping-pong, 16 MFMA/segment", 2000);
        bar_case<8, 32, 0>("8 waves ping-pong, 32 MFMA/segment", 1000);
        bar_case<8, 64, 0>("8 waves ping-pong, 64 MFMA/segment", 500);
        bar_case<8, 16, 1>("8 waves, 16 MFMA then barrier", 2000);
        bar_case<8, 64, 1>("8 waves, 64 MFMA then barrier", 500);
        bar_case<4, 16, 2>("4 waves, no barriers", 2000);
        bar_case<4, 32, 1>("4 waves, 32 MFMA then barrier", 1000);
        bar_case<4, 64, 1>("4 waves, 64 MFMA then barrier", 500);
        bar_case<4, 128, 1>("4 waves, 128 MFMA then barrier", 250);
        unsigned char* src;
        CK(hipMalloc(&src, (size_t)512 << 20));
        CK(hipMemset(src, 0, (size_t)512 << 20));
        seg_case<16, 0, 0>(src, 2000);
        seg_case<16, 0, 4>(src, 2000);
        seg_case<16, 0, 8>(src, 2000);
        seg_case<16, 0, 12>(src, 2000);
        seg_case<16, 1, 0>(src, 2000);
        seg_case<16, 2, 0>(src, 2000);
        seg_case<16, 4, 0>(src, 2000);
        seg_case<16, 2, 8>(src, 2000);
        seg_case<16, 2, 12>(src, 2000);
        seg_case<32, 0, 16>(src, 1000);
        seg_case<32, 4, 0>(src, 1000);
        seg_case<32, 4, 12>(src, 1000);
        seg_case<32, 4, 16>(src, 1000);
        seg_case<64, 8, 24>(src, 500);
        seg_case<0, 2, 8>(src, 2000);
        seg_case<0, 2, 0>(src, 2000);
        seg_case<0, 0, 8>(src, 2000);
        // v72's segment against the source pattern
        seg_case<32, 4, 12, 0>(src, 1000);
        seg_case<32, 4, 12, 1>(src, 1000);
        seg_case<32, 4, 12, 2>(src, 1000);
        seg_case<32, 4, 12, 3>(src, 1000);
        seg_case<0, 4, 12, 0>(src, 1000);
        seg_case<0, 4, 12, 1>(src, 1000);
        seg_case<0, 4, 12, 3>(src, 1000);
        seg_case<16, 2, 12, 1>(src, 2000);
        seg_case<16, 2, 12, 3>(src, 2000);
        return 0;
    }
    // p32run M N K epi xcd iters kind: plain launches for PMC passes. kind 0 v72 row-major A / W,
    // 1 v72 blocked A + W, 2 the v62 copy, 3 the shipped c_fc (v75: row-major A, blocked W,
    // balanced grid)
    if (argc > 1 && std::string(argv[1]) == "p32run") {
        const int M = atoi(argv[2]), N = atoi(argv[3]), K = atoi(argv[4]), epi = atoi(argv[5]), xcd = atoi(argv[6]);
        const int iters = atoi(argv[7]), kind = argc > 8 ? atoi(argv[8]) : 0;
        u16 *A, *W, *C;
        float* bias;
        CK(hipMalloc(&A, (size_t)(M + 256) * K * 2));
        CK(hipMalloc(&W, (size_t)N * K * 2));
        CK(hipMalloc(&C, (size_t)M * N * 2));
        CK(hipMalloc(&bias, (size_t)N * 4));
        fill_f16<<<1024, 256>>>(A, (size_t)(M + 256) * K, 1);
        fill_f16<<<1024, 256>>>(W, (size_t)N * K, 2);
        CK(hipMemset(bias, 0, N * 4));
        GemmArgs a{};
        a.A = A; a.W = W; a.bias = bias; a.C = C;
        a.M = M; a.N = N; a.K = K; a.ldc = N; a.xcd_n = xcd;
        const int ntiles = ((M + 255) / 256) * (N / 256), per = (ntiles + 255) / 256;
        const int grid = kind == 3 ? (ntiles + per - 1) / per : std::min(ntiles, 256);
        for (int i = 0; i < iters; ++i) {
            if (kind == 2) {
                if (epi) ppp_probe<F16, EPI_GELU, 0, false><<<grid, 512>>>(a, ntiles, nullptr);
                else ppp_probe<F16, EPI_STORE, 0, false><<<grid, 512>>>(a, ntiles, nullptr);
            } else if (kind == 1) {
                if (epi) gemm_p32_kernel<F16, EPI_GELU, true, true><<<grid, 512>>>(a, ntiles);
                else gemm_p32_kernel<F16, EPI_STORE, true, true><<<grid, 512>>>(a, ntiles);
            } else if (kind == 3) {
                if (epi) gemm_p32_kernel<F16, EPI_GELU, false, true><<<grid, 512>>>(a, ntiles);
                else gemm_p32_kernel<F16, EPI_STORE, false, true><<<grid, 512>>>(a, ntiles);
            } else {
                if (epi) gemm_p32_kernel<F16, EPI_GELU, false, false><<<grid, 512>>>(a, ntiles);
                else gemm_p32_kernel<F16, EPI_STORE, false, false><<<grid, 512>>>(a, ntiles);
            }
        }
        CK(hipDeviceSynchronize());
        printf("p32run done\n");
        return 0;
    }
    // p32 M N K epi xcd [balanced]: the shipped kernel (row-major A, blocked W, as c_fc / QKV run
    // it) with the stamp policy after ~2 s of plain launches: the per-phase cycle table of the
    // k-loop; then the ablations (P32Abl) and the plain kernel, best of 5 x 20 launches.
    if (argc > 1 && std::string(argv[1]) == "p32") {
        const int M = atoi(argv[2]), N = atoi(argv[3]), K = atoi(argv[4]), epi = atoi(argv[5]), xcd = atoi(argv[6]);
        const bool bal = argc > 7 && atoi(argv[7]) != 0;
        u16 *A, *W, *C;
        float* bias;
        CK(hipMalloc(&A, (size_t)(M + 256) * K * 2));
        CK(hipMalloc(&W, (size_t)N * K * 2));
        CK(hipMalloc(&C, (size_t)M * N * 2));
        CK(hipMalloc(&bias, (size_t)N * 4));
        fill_f16<<<1024, 256>>>(A, (size_t)(M + 256) * K, 1);
        fill_f16<<<1024, 256>>>(W, (size_t)N * K, 2);
        CK(hipMemset(bias, 0, N * 4));
        GemmArgs a{};
        a.A = A; a.W = W; a.bias = bias; a.C = C;
        a.M = M; a.N = N; a.K = K; a.ldc = N; a.xcd_n = xcd; a.blk_w = 1;
        const int ntiles = ((M + 255) / 256) * (N / 256), per = (ntiles + 255) / 256;
        const int grid = bal ? (ntiles + per - 1) / per : std::min(ntiles, 256);
        printf("p32 %dx%dx%d epi%d xcd%d: %d tiles on %d workgroups\n", M, N, K, epi, xcd, ntiles, grid);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        auto run = [&](const char* name, auto fn) {
            for (int i = 0; i < 5; ++i) fn();
            float best = 1e9f;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(e0));
                for (int i = 0; i < 20; ++i) fn();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms / 20);
            }
            printf("%-34s %7.2f us  %.0f TF/s\n", name, best * 1e3, 2.0 * M * N * K / (best * 1e-3) / 1e12);
        };
        {
            unsigned* tr;
            CK(hipMalloc(&tr, (size_t)grid * 8 * NST * 4));
            CK(hipMemset(tr, 0, (size_t)grid * 8 * NST * 4));
            CK(hipMemcpyToSymbol(HIP_SYMBOL(g_p32_trace), &tr, sizeof(tr)));
            CK(hipEventRecord(e0));
            float ms = 0.f;
            while (ms < 2000.f) {
                for (int i = 0; i < 100; ++i) {
                    if (epi) gemm_p32_kernel<F16, EPI_GELU, false, true><<<grid, 512>>>(a, ntiles);
                    else gemm_p32_kernel<F16, EPI_STORE, false, true><<<grid, 512>>>(a, ntiles);
                }
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
            }
            if (epi) gemm_p32_kernel<F16, EPI_GELU, false, true, false, 256, P32Stamp><<<grid, 512>>>(a, ntiles);
            else gemm_p32_kernel<F16, EPI_STORE, false, true, false, 256, P32Stamp><<<grid, 512>>>(a, ntiles);
            CK(hipDeviceSynchronize());
            std::vector<unsigned> t((size_t)grid * 8 * NST);
            CK(hipMemcpy(t.data(), tr, t.size() * 4, hipMemcpyDeviceToHost));
            auto u64 = [&](const unsigned* p, int i) { return (unsigned long long)p[i] | ((unsigned long long)p[i + 1] << 32); };
            auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? -1.0 : v[v.size() / 2]; };
            std::vector<double> clk, span;
            for (int g = 0; g < grid; ++g) {
                const unsigned* p = &t[(size_t)g * 8 * NST];
                clk.push_back((double)(u64(p, 4) - u64(p, 0)) / (double)(u64(p, 6) - u64(p, 2)) * 0.1);
                span.push_back((double)(u64(p, 6) - u64(p, 2)) * 0.01);
            }
            printf("stamped: in-kernel clock %.3f GHz (median), workgroup span %.2f us (median)\n", med(clk), med(span));
            const int nks = std::min(K / 32, 24);
            // slot of a stamp: [0] arrive R-barrier, [1] depart, [2] arrive M-barrier, [3] depart,
            // [4 + p] at() point p (0 issue, 1 vm wait, 2 epilogue, 3 reads, 4 -> 5 M lgkm, 5 -> 6 MFMA issue)
            auto slot = [&](int tix, int st, int k) { return 8 + tix * P32_TILE + st * P32_STEP + k; };
            // a phase = median over workgroups of stamp(b) - stamp(a) for one wave
            auto phase = [&](int wv, int tix, int st, int sa, int ka, int sb, int kb) {
                std::vector<double> v;
                for (int g = 0; g < grid; ++g) {
                    const unsigned* p = &t[((size_t)g * 8 + wv) * NST];
                    const unsigned x = p[slot(tix, sa, ka)], y = p[slot(tix, sb, kb)];
                    if (x && y) v.push_back((double)(unsigned)(y - x));
                }
                return med(v);
            };
            const char* names[] = {"R: staging issue", "R: vm wait (group 1)", "R: frag reads issue+drain / issue",
                                   "R: to barrier", "R: barrier wait", "M: lgkm drain", "M: MFMA issue",
                                   "M: vm wait (group 0) + to barrier", "M: barrier wait", "k-step"};
            for (int tix = 0; tix < 2; ++tix)
                for (int wv : {0, 4}) {
                    const bool g1 = wv >= 4;
                    double acc[10] = {0};
                    int nn = 0;
                    for (int st = 4; st < nks - 1; ++st) {
                        double ph[10];
                        ph[0] = phase(wv, tix, st - 1, st - 1, 3, st, 4);          // depart M(t-1) -> issue
                        ph[1] = g1 ? phase(wv, tix, st, st, 4, st, 5) : 0.0;      // issue -> vm wait
                        ph[2] = g1 ? phase(wv, tix, st, st, 5, st, 7) : phase(wv, tix, st, st, 4, st, 0);  // reads
                        ph[3] = g1 ? phase(wv, tix, st, st, 7, st, 0) : 0.0;
                        ph[4] = phase(wv, tix, st, st, 0, st, 1);
                        ph[5] = phase(wv, tix, st, st, 1, st, 8);
                        ph[6] = phase(wv, tix, st, st, 8, st, 9);
                        ph[7] = phase(wv, tix, st, st, 9, st, 2);
                        ph[8] = phase(wv, tix, st, st, 2, st, 3);
                        ph[9] = phase(wv, tix, st - 1, st - 1, 3, st, 3);
                        for (int k = 0; k < 10; ++k) acc[k] += ph[k];
                        ++nn;
                    }
                    printf("tile %d wave %d (group %d), steady steps 4..%d, cycles per k-step (median over WGs):\n", tix, wv, g1, nks - 2);
                    for (int k = 0; k < 10; ++k) printf("  %-36s %6.0f\n", names[k], acc[k] / nn);
                }
            CK(hipFree(tr));
        }
        for (int rep = 0; rep < 2; ++rep) {
#define P32RUN(NAME, HKT)                                                                          \
    run(NAME, [&] {                                                                                \
        if (epi) gemm_p32_kernel<F16, EPI_GELU, false, true, false, 256, HKT><<<grid, 512>>>(a, ntiles); \
        else gemm_p32_kernel<F16, EPI_STORE, false, true, false, 256, HKT><<<grid, 512>>>(a, ntiles);    \
    })
            P32RUN("shipped (A row-major, W blocked)", P32Abl<0>);
            P32RUN("ablation: no staging", P32Abl<7>);
            P32RUN("ablation: no MFMA", P32Abl<8>);
            P32RUN("ablation: no fragment reads", P32Abl<9>);
            P32RUN("ablation: no epilogue stores", P32Abl<3>);
#undef P32RUN
        }
        return 0;
    }
    // p32x M N K epi xcd: the 320 x 256 form (BM = 320, variant 77's balanced grid) against the
    // 256 x 256 one (variant 75), each with the ablation policies: which stream grows with BM
    if (argc > 1 && std::string(argv[1]) == "p32x") {
        const int M = atoi(argv[2]), N = atoi(argv[3]), K = atoi(argv[4]), epi = atoi(argv[5]), xcd = atoi(argv[6]);
        u16 *A, *W, *C;
        float* bias;
        CK(hipMalloc(&A, (size_t)(M + 320) * K * 2));
        CK(hipMalloc(&W, (size_t)N * K * 2));
        CK(hipMalloc(&C, (size_t)M * N * 2));
        CK(hipMalloc(&bias, (size_t)N * 4));
        fill_f16<<<1024, 256>>>(A, (size_t)(M + 320) * K, 1);
        fill_f16<<<1024, 256>>>(W, (size_t)N * K, 2);
        CK(hipMemset(bias, 0, N * 4));
        GemmArgs a{};
        a.A = A; a.W = W; a.bias = bias; a.C = C;
        a.M = M; a.N = N; a.K = K; a.ldc = N; a.xcd_n = xcd; a.blk_w = 1;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        auto run = [&](const char* name, double tiles, auto fn) {
            for (int i = 0; i < 5; ++i) fn();
            float best = 1e9f;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(e0));
                for (int i = 0; i < 20; ++i) fn();
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms / 20);
            }
            printf("%-40s %7.2f us  %.0f TF/s  %.2f us per tile-round\n", name, best * 1e3,
                   2.0 * M * N * K / (best * 1e-3) / 1e12, best * 1e3 / tiles);
        };
        for (int bm : {256, 320}) {
            const int ntiles = ((M + bm - 1) / bm) * (N / 256), per = (ntiles + 255) / 256;
            const int grid = (ntiles + per - 1) / per;
            printf("BM %d: %d tiles on %d workgroups (%d per workgroup)\n", bm, ntiles, grid, per);
#define P32X(NAME, BMV, HKT)                                                                               \
    run(NAME, per, [&] {                                                                                    \
        if (epi) gemm_p32_kernel<F16, EPI_GELU, false, true, false, BMV, HKT><<<grid, 512>>>(a, ntiles);  \
        else gemm_p32_kernel<F16, EPI_STORE, false, true, false, BMV, HKT><<<grid, 512>>>(a, ntiles);     \
    })
            if (bm == 256) {
                P32X("  BM 256 shipped", 256, P32Abl<0>);
                P32X("  BM 256 no staging", 256, P32Abl<7>);
                P32X("  BM 256 no MFMA", 256, P32Abl<8>);
                P32X("  BM 256 no fragment reads", 256, P32Abl<9>);
                P32X("  BM 256 no epilogue stores", 256, P32Abl<3>);
            } else {
                P32X("  BM 320 shipped", 320, P32Abl<0>);
                P32X("  BM 320 no staging", 320, P32Abl<7>);
                P32X("  BM 320 no MFMA", 320, P32Abl<8>);
                P32X("  BM 320 no fragment reads", 320, P32Abl<9>);
                P32X("  BM 320 no epilogue stores", 320, P32Abl<3>);
            }
#undef P32X
        }
        return 0;
    }
    if (argc < 6) {
        fprintf(stderr, "usage: gemm_probe M N K epi xcd [iters] [grid]\n");
        return 2;
    }
    const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]), epi = atoi(argv[4]), xcd = atoi(argv[5]);
    const int iters = argc > 6 ? atoi(argv[6]) : 50;
    int ncu = 256;
    {
        int d = 0;
        CK(hipGetDevice(&d));
        CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, d));
    }
    const int gridmax = argc > 7 ? atoi(argv[7]) : ncu;
    if (N % 256 || K % 128 || N > 4096 || M <= 0) {
        fprintf(stderr, "shape: N %% 256, K %% 128, N <= 4096\n");
        return 2;
    }
    u16 *A, *W, *C;
    float *bias, *R;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&W, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMalloc(&R, (size_t)M * N * 4));
    CK(hipMalloc(&bias, (size_t)N * 4));
    fill_f16<<<1024, 256>>>(A, (size_t)M * K, 1);
    fill_f16<<<1024, 256>>>(W, (size_t)N * K, 2);
    {
        std::vector<float> b(N);
        for (int i = 0; i < N; ++i) b[i] = 0.01f * (float)((i * 37) % 101 - 50);
        CK(hipMemcpy(bias, b.data(), N * 4, hipMemcpyHostToDevice));
    }
    GemmArgs a{};
    a.A = A; a.W = W; a.bias = bias; a.C = C;
    a.M = M; a.N = N; a.K = K; a.ldc = N;
    a.xcd_n = xcd;
    const int ntiles = ((M + 255) / 256) * (N / 256);
    const int grid = std::min(ntiles, gridmax);
    unsigned* tr = nullptr;
    CK(hipMalloc(&tr, (size_t)grid * 8 * NST * 4));
    CK(hipMemset(tr, 0, (size_t)grid * 8 * NST * 4));

    // correctness of the plain build
    LaunchFn plain = epi ? pick<1>(0, false) : pick<0>(0, false);
    plain(a, grid, ntiles, nullptr);
    ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(A, W, bias, R, M, N, K, epi);
    CK(hipDeviceSynchronize());
    {
        std::vector<u16> c((size_t)M * N);
        std::vector<float> r((size_t)M * N);
        CK(hipMemcpy(c.data(), C, c.size() * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r.data(), R, r.size() * 4, hipMemcpyDeviceToHost));
        double maxerr = 0, maxref = 0;
        for (size_t i = 0; i < c.size(); ++i) {
            const double v = (double)(float)__builtin_bit_cast(_Float16, c[i]);
            maxerr = std::max(maxerr, std::fabs(v - r[i]));
            maxref = std::max(maxref, (double)std::fabs(r[i]));
        }
        printf("check %dx%dx%d epi%d: max|err| %.3e max|ref| %.3e rel %.2e %s\n", M, N, K, epi, maxerr, maxref,
               maxerr / maxref, maxerr / maxref < 4e-3 ? "OK" : "FAIL");
        if (!(maxerr / maxref < 4e-3)) return 1;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double flop = 2.0 * M * N * K;
    for (int abl : {0, 3, 7, 8}) {
        LaunchFn f = epi ? pick<1>(abl, false) : pick<0>(abl, false);
        for (int i = 0; i < 5; ++i) f(a, grid, ntiles, nullptr);
        float best = 1e9f, sum = 0.f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            for (int i = 0; i < iters; ++i) f(a, grid, ntiles, nullptr);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= iters;
            best = std::min(best, ms);
            sum += ms;
        }
        printf("abl %d: best %.2f us avg %.2f us  %.0f TF/s (%.3f of 2516.6)\n", abl, best * 1e3, sum / 5 * 1e3,
               flop / (best * 1e-3) / 1e12, flop / (best * 1e-3) / 1e12 / 2516.6);
    }
    // stamped launch after ~2 s of back-to-back plain launches (clock settled)
    {
        CK(hipEventRecord(e0));
        float ms = 0;
        int n = 0;
        while (ms < 2000.f) {
            for (int i = 0; i < 100; ++i) plain(a, grid, ntiles, nullptr);
            n += 100;
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
        }
        LaunchFn s = epi ? pick<1>(0, true) : pick<0>(0, true);
        s(a, grid, ntiles, tr);
        CK(hipDeviceSynchronize());
        printf("warm-up %d launches %.0f ms (%.2f us each)\n", n, ms, ms * 1e3 / n);
    }
    std::vector<unsigned> t((size_t)grid * 8 * NST);
    CK(hipMemcpy(t.data(), tr, t.size() * 4, hipMemcpyDeviceToHost));
    auto u64 = [&](const unsigned* p, int i) { return (unsigned long long)p[i] | ((unsigned long long)p[i + 1] << 32); };
    // clock per workgroup (wave 0)
    std::vector<double> clk, dur;
    unsigned long long rt0 = ~0ull;
    for (int g = 0; g < grid; ++g) rt0 = std::min(rt0, u64(&t[(size_t)g * 8 * NST], 2));
    for (int g = 0; g < grid; ++g) {
        const unsigned* p = &t[(size_t)g * 8 * NST];
        const double dm = (double)(u64(p, 4) - u64(p, 0)), dr = (double)(u64(p, 6) - u64(p, 2));
        clk.push_back(dm / dr * 0.1);
        dur.push_back(dr * 0.01);
    }
    std::sort(clk.begin(), clk.end());
    std::sort(dur.begin(), dur.end());
    printf("in-kernel clock (GHz): min %.3f median %.3f max %.3f; workgroup span (us): min %.2f median %.2f max %.2f\n",
           clk.front(), clk[clk.size() / 2], clk.back(), dur.front(), dur[dur.size() / 2], dur.back());
    // start skew
    {
        std::vector<double> s0;
        for (int g = 0; g < grid; ++g) s0.push_back((u64(&t[(size_t)g * 8 * NST], 2) - rt0) * 0.01);
        std::sort(s0.begin(), s0.end());
        printf("workgroup start skew (us): median %.2f max %.2f\n", s0[s0.size() / 2], s0.back());
    }
    // per barrier interval e of k-tile kt, one wave: work = arrival(e) - departure(e - 1) (its
    // own instruction stream), wait = departure(e) - arrival(e) (parked at the barrier); medians
    // over workgroups. Only tile 0 and 1 (tile 2 exists on few workgroups of these shapes).
    const int nkt = std::min(K / 64, ST_KT);
    auto med = [](std::vector<double>& v) { std::sort(v.begin(), v.end()); return v.empty() ? -1.0 : v[v.size() / 2]; };
    for (int tix = 0; tix < 2; ++tix) {
        for (int wv : {0, 4, 1, 5}) {
            printf("tile %d wave %d (group %d): per k-tile [8 barrier intervals] work/wait cycles\n", tix, wv, wv / 4);
            double sw = 0, sx = 0;
            int nn = 0;
            for (int kt = 0; kt < nkt; ++kt) {
                printf("  kt %2d:", kt);
                double tw = 0, tx = 0;
                for (int e = 0; e < 8; ++e) {
                    std::vector<double> w, x;
                    for (int g = 0; g < grid; ++g) {
                        const unsigned* p = &t[((size_t)g * 8 + wv) * NST];
                        const int d1 = 8 + tix * ST_PER_TILE + 8 * kt + e, a1 = d1 + 8 * ST_KT;
                        const int d0 = (e > 0 || kt > 0) ? d1 - 1 : -1;
                        if (!p[d1] || !p[a1]) continue;
                        x.push_back((double)(unsigned)(p[d1] - p[a1]));
                        if (d0 >= 0 && p[d0]) w.push_back((double)(unsigned)(p[a1] - p[d0]));
                    }
                    const double mw = med(w), mx = med(x);
                    printf(" %4.0f/%-4.0f", mw, mx);
                    if (mw > 0) tw += mw;
                    if (mx > 0) tx += mx;
                }
                printf(" | %5.0f/%-5.0f\n", tw, tx);
                if (kt >= 2 && kt + 1 < nkt) { sw += tw; sx += tx; ++nn; }
            }
            if (nn) printf("  steady k-tile (kt 2..%d): work %.0f + wait %.0f = %.0f cyc\n", nkt - 2, sw / nn, sx / nn, (sw + sx) / nn);
            std::vector<double> ep, kl;
            for (int g = 0; g < grid; ++g) {
                const unsigned* p = &t[((size_t)g * 8 + wv) * NST];
                const int b = 8 + tix * ST_PER_TILE;
                const unsigned e0s = p[b + 16 * ST_KT], e1s = p[b + 16 * ST_KT + 1];
                if (!e0s || !e1s) continue;
                ep.push_back((double)(unsigned)(e1s - e0s));
                if (p[b]) kl.push_back((double)(unsigned)(e0s - p[b]));
            }
            printf("  epilogue %.0f cyc, k-loop (first barrier -> epilogue) %.0f cyc (n=%zu)\n", med(ep), med(kl), ep.size());
        }
    }
    return 0;
}
