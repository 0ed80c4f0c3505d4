// The classifier head, all fp32 (a 1e-3-relative logit bar leaves no room for 16-bit here):
//   f      = ln_post(x[:, 0, :]) @ proj                    [3p] VisionTransformer.forward tail
//   f_hat  = f / ||f||                                      main.py:205, main.py:445, main.py:504
//   logits = 100 * f_hat @ T^T                              main.py:208, main.py:456, main.py:506
//   probs  = softmax(logits) inside each label segment      (detector 40 | styles | ... )
//   top-k  = topk(min(5, n)) per segment                    main.py:211, main.py:457, main.py:507
// T rows are the cached, already L2-normalised text features (main.py:179-182, 296-311); the
// library keeps them transposed (Tt [E][Cpad]) so column tiles load coalesced.
//
// These kernels move a few MB and do ~0.3 GFLOP per batch of 256, so they are bound by latency,
// not bandwidth (the first version ran 134 us per batch, measured: one global round trip per
// 64-deep chunk, three passes over every LayerNorm row, and 18 serially dependent cross-lane
// shuffles per top-k slot on one wave per image). Here:
//  * both products (B x D x E and B x E x C) use 16-image x 64-column tiles whose weight chunks
//    are prefetched into registers two chunks ahead of the one being multiplied from LDS;
//  * a row (LayerNorm input, feature vector) is loaded with all its loads in flight at once and
//    reduced from registers;
//  * softmax + top-k runs one wave per (image, segment), all segments of an image in parallel.
// Per-image results never depend on the batch size or the image's position in it.
#include "common.h"

namespace clipvit {

constexpr int HR = 16;     // images per workgroup
constexpr int HW = 8;      // waves per workgroup (two per SIMD: one wave's LDS / global latency
                           // hides behind the other's FMAs)
constexpr int HT = 64 * HW;
constexpr int HK = 128;    // reduction chunk (rows of the weight operand per LDS fill)
constexpr int HMAXD = 20;  // max row length / 64 held in registers (width <= 1280)

// Stage rows [b0, b0 + 16) of a [*, ld] fp32 matrix (row stride `stride` floats) into LDS
// [16][n], optionally LayerNorm-ed (gamma, beta) or L2-normalised; one wave per row, all of a
// row's loads issued before any is used. Rows >= B are zero.
template <int MODE>  // 0 LayerNorm, 1 L2 normalise
__device__ __forceinline__ void stage_rows(const float* __restrict__ src, size_t stride, int b0, int B,
                                           int n, const float* __restrict__ gm,
                                           const float* __restrict__ bt, float* dst,
                                           float* __restrict__ norm_out) {
    // the wave's HR / HW rows: every load of every row is issued before the first reduction (one
    // memory round trip per wave instead of one per row)
    constexpr int RW = HR / HW;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nv = n >> 6;
    float v[RW][HMAXD];
#pragma unroll
    for (int rr = 0; rr < RW; ++rr) {
        const int b = min(b0 + wave + HW * rr, B - 1);  // rows past B: clamped load, zero row below
        const float* r = src + (size_t)b * stride;
#pragma unroll
        for (int j = 0; j < HMAXD; ++j) {  // unconditional loads (clamped address), then select
            const float t = r[lane + 64 * min(j, nv - 1)];
            v[rr][j] = j < nv ? t : 0.f;
        }
    }
#pragma unroll
    for (int rr = 0; rr < RW; ++rr) {
        const int i = wave + HW * rr, b = b0 + i;
        float* d = dst + i * (n + 4);  // rows padded by 4 floats: the product's 4 image reads hit distinct banks
        if (b >= B) {
            for (int c = lane; c < n; c += 64) d[c] = 0.f;
            continue;
        }
        if constexpr (MODE == 0) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < HMAXD; ++j) s += v[rr][j];
            const float mean = wave_sum(s) / n;
            float q = 0.f;
#pragma unroll
            for (int j = 0; j < HMAXD; ++j)
                if (j < nv) q += (v[rr][j] - mean) * (v[rr][j] - mean);
            const float rstd = rsqrtf(wave_sum(q) / n + 1e-5f);
#pragma unroll
            for (int j = 0; j < HMAXD; ++j)
                if (j < nv) {
                    const int c = lane + 64 * j;
                    d[c] = (v[rr][j] - mean) * rstd * gm[c] + bt[c];
                }
        } else {
            float q = 0.f;
#pragma unroll
            for (int j = 0; j < HMAXD; ++j) q += v[rr][j] * v[rr][j];
            const float inv = 1.0f / sqrtf(wave_sum(q));
#pragma unroll
            for (int j = 0; j < HMAXD; ++j)
                if (j < nv) {
                    const int c = lane + 64 * j;
                    d[c] = v[rr][j] * inv;
                    if (norm_out) norm_out[(size_t)b * n + c] = v[rr][j] * inv;
                }
        }
    }
}

// P = xs[16][K] @ W[K][col0 .. col0 + TC)  (K % 128 == 0; TC = 64 or 32 output columns per
// workgroup), xs in LDS (row stride K + 4) staged by `stage()`, which runs while the first two
// weight chunks are in flight. Weight chunks (128 x TC) go global -> registers two chunks ahead
// of the multiply, registers -> LDS ws (row stride TC + 4). Wave w multiplies k-rows
// [16 w, 16 w + 16) of every chunk into a full 16 x TC partial tile (lane: images 4 (lane >> 4)
// .. + 3, columns CPL (lane & 15) .. + CPL - 1, CPL = TC / 16); the HW partials are summed in a
// fixed order at the end. On return, threads tid < 4 TC hold in red[i] the output (image
// tid / (TC / 4), columns 4 (tid % (TC / 4)) + i). Every output element sees the same
// arithmetic in the same order for either TC (bit-identical results).
template <int TC, typename Stage>
__device__ __forceinline__ void tile_product(const float* xs, int K, const float* __restrict__ W, int ldw,
                                             int col0, float* ws, float (&red)[4], int tid, Stage&& stage) {
    constexpr int KW = HK / HW;      // k-rows of a chunk per wave
    constexpr int CPL = TC / 16;     // output columns per lane
    constexpr int TPR = TC / 4;      // threads per weight row (one float4 each)
    constexpr int RPP = HT / TPR;    // weight rows per load pass
    constexpr int NP = HK / RPP;     // load passes per chunk (4 for TC = 64, 2 for 32)
    constexpr int WS = TC + 4;       // ws row stride (floats)
    static_assert(TC == 64 || TC == 32, "column tile");
    const int lane = tid & 63, wave = tid >> 6;
    const int ig = lane >> 4, cg = lane & 15;
    const int lr = tid / TPR, lc = (tid % TPR) * 4;
    const int nc = K / HK;
    const int xstride = K + 4;
    float acc[4][CPL] = {};
    // two register chunks of NP float4 (named scalars: an array here ends up in scratch)
    float4 a0, a1, a2, a3, b0, b1, b2, b3;
    const size_t lpass = (size_t)RPP * ldw;
#define HEAD_LOAD(x0, x1, x2, x3, k0)                                      \
    {                                                                      \
        const float* p_ = W + (size_t)((k0) + lr) * ldw + col0 + lc;       \
        x0 = *(const float4*)p_;                                           \
        x1 = *(const float4*)(p_ + lpass);                                 \
        if constexpr (NP == 4) {                                           \
            x2 = *(const float4*)(p_ + 2 * lpass);                         \
            x3 = *(const float4*)(p_ + 3 * lpass);                         \
        }                                                                  \
    }
#define HEAD_PUT(x0, x1, x2, x3)                                           \
    {                                                                      \
        float* q_ = ws + lr * WS + lc;                                     \
        *(float4*)q_ = x0;                                                 \
        *(float4*)(q_ + RPP * WS) = x1;                                    \
        if constexpr (NP == 4) {                                           \
            *(float4*)(q_ + 2 * RPP * WS) = x2;                            \
            *(float4*)(q_ + 3 * RPP * WS) = x3;                            \
        }                                                                  \
    }
    auto mul = [&](int k0) {
        const float* xr = xs + (4 * ig) * xstride + k0 + KW * wave;
        const float* wr = ws + (KW * wave) * WS + CPL * cg;
#pragma unroll
        for (int k = 0; k < KW; k += 4) {
            float4 x[4];
            float w[4][CPL];
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = *(const float4*)(xr + i * xstride + k);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if constexpr (CPL == 4) {
                    const float4 t = *(const float4*)(wr + (k + j) * WS);
                    w[j][0] = t.x; w[j][1] = t.y; w[j][2] = t.z; w[j][3] = t.w;
                } else {
                    const float2 t = *(const float2*)(wr + (k + j) * WS);
                    w[j][0] = t.x; w[j][1] = t.y;
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float xv[4] = {x[i].x, x[i].y, x[i].z, x[i].w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int c = 0; c < CPL; ++c) acc[i][c] += xv[j] * w[j][c];
            }
        }
    };
    HEAD_LOAD(a0, a1, a2, a3, 0);
    if (nc > 1) HEAD_LOAD(b0, b1, b2, b3, HK);
    stage();
    for (int c = 0; c < nc; c += 2) {
        __syncthreads();  // xs staged (first pass) / previous chunk's reads done
        HEAD_PUT(a0, a1, a2, a3);
        __syncthreads();
        if (c + 2 < nc) HEAD_LOAD(a0, a1, a2, a3, (c + 2) * HK);
        mul(c * HK);
        if (c + 1 >= nc) break;
        __syncthreads();
        HEAD_PUT(b0, b1, b2, b3);
        __syncthreads();
        if (c + 3 < nc) HEAD_LOAD(b0, b1, b2, b3, (c + 3) * HK);
        mul((c + 1) * HK);
    }
#undef HEAD_LOAD
#undef HEAD_PUT
    // sum the HW per-wave partial tiles (fixed order) through LDS
    __syncthreads();
    float* part = ws;  // [HW waves][16 images][TC columns]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < CPL; ++c) part[wave * 16 * TC + (4 * ig + i) * TC + CPL * cg + c] = acc[i][c];
    __syncthreads();
    const int img = (tid / TPR) & 15, cq = (tid % TPR) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) red[i] = 0.f;
#pragma unroll
    for (int w = 0; w < HW; ++w) {
        const float4 v = *(const float4*)(part + w * 16 * TC + img * TC + cq);
        red[0] += v.x; red[1] += v.y; red[2] += v.z; red[3] += v.w;
    }
}

// grid (ceil(B/16), E/TC), HT threads.
template <int TC>
__global__ __launch_bounds__(HT) void cls_ln_proj_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ gm,
                                                          const float* __restrict__ bt,
                                                          const float* __restrict__ proj,
                                                          float* __restrict__ f, int B, int N,
                                                          int D, int E) {
    extern __shared__ __attribute__((aligned(16))) float sm[];  // [16][D + 4] + [128][TC + 4]
    float* ys = sm;
    float* ws = sm + HR * (D + 4);
    const int tid = threadIdx.x;
    const int b0 = blockIdx.x * HR, col0 = blockIdx.y * TC;
    float red[4];
    tile_product<TC>(ys, D, proj, E, col0, ws, red, tid, [&]() {  // CLS token = row 0 of each image
        stage_rows<0>(x, (size_t)N * D, b0, B, D, gm, bt, ys, nullptr);
    });
    const int b = b0 + tid / (TC / 4);
    if (tid < 4 * TC && b < B)
        *(float4*)(f + (size_t)b * E + col0 + (tid % (TC / 4)) * 4) = make_float4(red[0], red[1], red[2], red[3]);
}

// grid (ceil(B/16), Cpad/TC), HT threads.
template <int TC>
__global__ __launch_bounds__(HT) void logits_kernel(const float* __restrict__ f,
                                                     const float* __restrict__ Tt,
                                                     float* __restrict__ emb_norm,
                                                     float* __restrict__ logits, int B, int E,
                                                     int C, int Cpad) {
    extern __shared__ __attribute__((aligned(16))) float sm[];  // [16][E + 4] + [128][TC + 4]
    float* fs = sm;
    float* ws = sm + HR * (E + 4);
    const int tid = threadIdx.x;
    const int b0 = blockIdx.x * HR, col0 = blockIdx.y * TC;
    float red[4];
    tile_product<TC>(fs, E, Tt, Cpad, col0, ws, red, tid, [&]() {
        stage_rows<1>(f, (size_t)E, b0, B, E, nullptr, nullptr, fs, blockIdx.y == 0 ? emb_norm : nullptr);
    });
    const int b = b0 + tid / (TC / 4), c = col0 + (tid % (TC / 4)) * 4;
    if (tid < 4 * TC && b < B) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (c + i < C) logits[(size_t)b * C + c + i] = 100.0f * red[i];
    }
}

// One workgroup per image, one wave per label segment (segments beyond the wave count loop):
// the image's logits row is staged in LDS, then each wave computes its segment's max / sum /
// probabilities and top-min(5, n) (ties -> lower index, like a stable sort) from LDS.
constexpr int SM_WAVES = 8;
__global__ __launch_bounds__(64 * SM_WAVES) void seg_softmax_topk_kernel(
    const float* __restrict__ logits, float* __restrict__ probs, int* __restrict__ top_idx,
    float* __restrict__ top_prob, const int* __restrict__ seg_off, int nseg, int B, int C) {
    extern __shared__ __attribute__((aligned(16))) float lr[];  // [C]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x;
    const float* src = logits + (size_t)b * C;
    for (int c = threadIdx.x; c < C; c += 64 * SM_WAVES) lr[c] = src[c];
    __syncthreads();
    for (int sg = wave; sg < nseg; sg += SM_WAVES) {
        const int s0 = seg_off[sg], s1 = seg_off[sg + 1], n = s1 - s0;
        float m = -INFINITY;
        for (int c = s0 + lane; c < s1; c += 64) m = fmaxf(m, lr[c]);
        m = wave_max(m);
        float sum = 0.f;
        for (int c = s0 + lane; c < s1; c += 64) sum += expf(lr[c] - m);
        sum = wave_sum(sum);
        const float inv = 1.0f / sum;
        if (probs)
            for (int c = s0 + lane; c < s1; c += 64) probs[(size_t)b * C + c] = expf(lr[c] - m) * inv;
        if (!top_idx && !top_prob) continue;
        const int k = n < 5 ? n : 5;
        int chosen[5] = {-1, -1, -1, -1, -1};
        for (int kk = 0; kk < 5; ++kk) {
            int bi = -1;
            float bv = -INFINITY;
            if (kk < k) {
                for (int c = s0 + lane; c < s1; c += 64) {
                    bool used = false;
#pragma unroll
                    for (int u = 0; u < 5; ++u) used |= (chosen[u] == c);
                    const float v = lr[c];
                    if (!used && (bi < 0 || v > bv)) { bv = v; bi = c; }
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) {
                    const float ov = __shfl_xor(bv, o, 64);
                    const int oi = __shfl_xor(bi, o, 64);
                    if (oi >= 0 && (bi < 0 || ov > bv || (ov == bv && oi < bi))) { bv = ov; bi = oi; }
                }
                chosen[kk] = bi;
            }
            if (lane == 0) {
                const size_t o = ((size_t)b * nseg + sg) * 5 + kk;
                if (top_idx) top_idx[o] = kk < k ? bi - s0 : -1;
                if (top_prob) top_prob[o] = kk < k ? expf(bv - m) * inv : 0.f;
            }
        }
    }
}

template <int TC>
static void cls_ln_proj_t(hipStream_t s, const float* x, const float* g, const float* b, const float* proj,
                          float* f, int B, int N, int D, int E) {
    static const bool attr = hipFuncSetAttribute((const void*)cls_ln_proj_kernel<TC>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024) == hipSuccess;
    (void)attr;
    dim3 grid((B + HR - 1) / HR, E / TC), block(HT);
    const size_t lds = (HR * (D + 4) + HK * (TC + 4)) * sizeof(float);
    cls_ln_proj_kernel<TC><<<grid, block, lds, s>>>(x, g, b, proj, f, B, N, D, E);
}

template <int TC>
static void logits_t(hipStream_t s, const float* f, const float* Tt, float* emb_norm, float* logits, int B,
                     int E, int C, int Cpad) {
    static const bool attr = hipFuncSetAttribute((const void*)logits_kernel<TC>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024) == hipSuccess;
    (void)attr;
    dim3 grid((B + HR - 1) / HR, Cpad / TC), block(HT);
    const size_t lds = (HR * (E + 4) + HK * (TC + 4)) * sizeof(float);
    logits_kernel<TC><<<grid, block, lds, s>>>(f, Tt, emb_norm, logits, B, E, C, Cpad);
}

// tc = output columns per workgroup (64 or 32; 32 doubles the workgroups of the small-batch
// grids, the arithmetic per output element is the same)
void launch_cls_ln_proj(hipStream_t s, const float* x, const float* g, const float* b,
                        const float* proj, float* f, int B, int N, int D, int E, int tc) {
    if (tc == 32) cls_ln_proj_t<32>(s, x, g, b, proj, f, B, N, D, E);
    else cls_ln_proj_t<64>(s, x, g, b, proj, f, B, N, D, E);
}

void launch_logits(hipStream_t s, const float* f, const float* Tt, float* emb_norm, float* logits,
                   int B, int E, int C, int Cpad, int tc) {
    if (tc == 32) logits_t<32>(s, f, Tt, emb_norm, logits, B, E, C, Cpad);
    else logits_t<64>(s, f, Tt, emb_norm, logits, B, E, C, Cpad);
}

void launch_seg_softmax_topk(hipStream_t s, const float* logits, float* probs, int* top_idx,
                             float* top_prob, const int* seg_off, int nseg, int B, int C) {
    seg_softmax_topk_kernel<<<B, 64 * SM_WAVES, C * sizeof(float), s>>>(logits, probs, top_idx, top_prob,
                                                                      seg_off, nseg, B, C);
}

}  // namespace clipvit
