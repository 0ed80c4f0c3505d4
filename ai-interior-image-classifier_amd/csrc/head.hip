// The classifier head, all fp32 (a 1e-3-relative logit bar leaves no room for 16-bit here):
//   f      = ln_post(x[:, 0, :]) @ proj                    [3p] VisionTransformer.forward tail
//   f_hat  = f / ||f||                                      main.py:205, main.py:445, main.py:504
//   logits = 100 * f_hat @ T^T                              main.py:208, main.py:456, main.py:506
//   probs  = softmax(logits) inside each label segment      (detector 40 | styles | ... )
//   top-k  = topk(min(5, n)) per segment                    main.py:211, main.py:457, main.py:507
// T rows are the cached, already L2-normalised text features (main.py:179-182, 296-311); the
// library keeps them transposed (Tt [E][Cpad]) so column tiles load coalesced.
//
// Both matrix products are small (B x 768 x 512 and B x 512 x 437): each workgroup computes a
// 16-image x 64-column tile, streaming the weight operand through LDS in 64-deep chunks with
// float4 loads (no per-iteration global-load latency), 4 images x 1 column per thread.
#include "common.h"

namespace clipvit {

constexpr int HR = 16;   // images per workgroup
constexpr int HK = 64;   // reduction chunk

// acc[i] += sum_k X[ib + i][k] * W[k][col]  for k in [0, K), X in LDS [HR][K], W global [K][ldw]
__device__ __forceinline__ void tile_accumulate(const float* __restrict__ xs, int K,
                                                const float* __restrict__ W, int ldw, int col0,
                                                float* ws, float (&acc)[4], int tid) {
    const int tx = tid & 63, ib = (tid >> 6) * 4;
    for (int k0 = 0; k0 < K; k0 += HK) {
        __syncthreads();
        // 64 x 64 chunk of W: thread loads 4 float4 (rows k0 + (tid >> 4) + 16 j, cols 4 (tid & 15))
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = (tid >> 4) + 16 * j, c = (tid & 15) * 4;
            *(float4*)(ws + r * 68 + c) = *(const float4*)(W + (size_t)(k0 + r) * ldw + col0 + c);
        }
        __syncthreads();
#pragma unroll 16
        for (int k = 0; k < HK; ++k) {
            const float w = ws[k * 68 + tx];
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] += xs[(ib + i) * K + k0 + k] * w;
        }
    }
}

// grid (ceil(B/16), E/64), 256 threads.
__global__ __launch_bounds__(256) void cls_ln_proj_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ gm,
                                                          const float* __restrict__ bt,
                                                          const float* __restrict__ proj,
                                                          float* __restrict__ f, int B, int N,
                                                          int D, int E) {
    extern __shared__ __attribute__((aligned(16))) float sm[];  // [16][D] + [64][68]
    float* ys = sm;
    float* ws = sm + HR * D;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b0 = blockIdx.x * HR;
    for (int i = wave; i < HR; i += 4) {  // LayerNorm of the CLS rows (one wave per row)
        const int b = b0 + i;
        float* yr = ys + i * D;
        if (b >= B) {
            for (int c = lane; c < D; c += 64) yr[c] = 0.f;
            continue;
        }
        const float* xr = x + (size_t)b * N * D;  // CLS token = row 0 of the image
        float s = 0.f;
        for (int c = lane; c < D; c += 64) s += xr[c];
        const float mean = wave_sum(s) / D;
        float q = 0.f;
        for (int c = lane; c < D; c += 64) {
            const float d = xr[c] - mean;
            q += d * d;
        }
        const float rstd = rsqrtf(wave_sum(q) / D + 1e-5f);
        for (int c = lane; c < D; c += 64) yr[c] = (xr[c] - mean) * rstd * gm[c] + bt[c];
    }
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int col0 = blockIdx.y * 64;
    tile_accumulate(ys, D, proj, E, col0, ws, acc, tid);
    const int ib = wave * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int b = b0 + ib + i;
        if (b < B) f[(size_t)b * E + col0 + lane] = acc[i];
    }
}

// grid (ceil(B/16), Cpad/64), 256 threads.
__global__ __launch_bounds__(256) void logits_kernel(const float* __restrict__ f,
                                                     const float* __restrict__ Tt,
                                                     float* __restrict__ emb_norm,
                                                     float* __restrict__ logits, int B, int E,
                                                     int C, int Cpad) {
    extern __shared__ __attribute__((aligned(16))) float sm[];  // [16][E] + [64][68]
    float* fs = sm;
    float* ws = sm + HR * E;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b0 = blockIdx.x * HR;
    for (int i = wave; i < HR; i += 4) {
        const int b = b0 + i;
        float* fr = fs + i * E;
        if (b >= B) {
            for (int c = lane; c < E; c += 64) fr[c] = 0.f;
            continue;
        }
        const float* src = f + (size_t)b * E;
        float q = 0.f;
        for (int c = lane; c < E; c += 64) q += src[c] * src[c];
        const float inv = 1.0f / sqrtf(wave_sum(q));
        for (int c = lane; c < E; c += 64) {
            const float v = src[c] * inv;
            fr[c] = v;
            if (emb_norm && blockIdx.y == 0) emb_norm[(size_t)b * E + c] = v;
        }
    }
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int col0 = blockIdx.y * 64;
    tile_accumulate(fs, E, Tt, Cpad, col0, ws, acc, tid);
    const int c = col0 + lane, ib = wave * 4;
    if (c < C) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int b = b0 + ib + i;
            if (b < B) logits[(size_t)b * C + c] = 100.0f * acc[i];
        }
    }
}

// One wave per image; the image's logits row is staged in LDS once, then every segment's
// max / sum / top-min(5, n) (ties -> lower index, like a stable sort) runs from LDS.
constexpr int SM_WAVES = 4;
__global__ __launch_bounds__(64 * SM_WAVES) void seg_softmax_topk_kernel(
    const float* __restrict__ logits, float* __restrict__ probs, int* __restrict__ top_idx,
    float* __restrict__ top_prob, const int* __restrict__ seg_off, int nseg, int B, int C) {
    extern __shared__ __attribute__((aligned(16))) float rows[];  // [SM_WAVES][C]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = blockIdx.x * SM_WAVES + wave;
    if (b >= B) return;
    float* lr = rows + wave * C;
    const float* src = logits + (size_t)b * C;
    for (int c = lane; c < C; c += 64) lr[c] = src[c];
    __builtin_amdgcn_s_waitcnt(0);  // own wave's LDS writes visible to its own later reads
    for (int sg = 0; sg < nseg; ++sg) {
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

void launch_cls_ln_proj(hipStream_t s, const float* x, const float* g, const float* b,
                        const float* proj, float* f, int B, int N, int D, int E) {
    static const bool attr = hipFuncSetAttribute((const void*)cls_ln_proj_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024) == hipSuccess;
    (void)attr;
    dim3 grid((B + HR - 1) / HR, E / 64), block(256);
    const size_t lds = (HR * D + 64 * 68) * sizeof(float);
    cls_ln_proj_kernel<<<grid, block, lds, s>>>(x, g, b, proj, f, B, N, D, E);
}

void launch_logits(hipStream_t s, const float* f, const float* Tt, float* emb_norm, float* logits,
                   int B, int E, int C, int Cpad) {
    static const bool attr = hipFuncSetAttribute((const void*)logits_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024) == hipSuccess;
    (void)attr;
    dim3 grid((B + HR - 1) / HR, Cpad / 64), block(256);
    const size_t lds = (HR * E + 64 * 68) * sizeof(float);
    logits_kernel<<<grid, block, lds, s>>>(f, Tt, emb_norm, logits, B, E, C, Cpad);
}

void launch_seg_softmax_topk(hipStream_t s, const float* logits, float* probs, int* top_idx,
                             float* top_prob, const int* seg_off, int nseg, int B, int C) {
    const int blocks = (B + SM_WAVES - 1) / SM_WAVES;
    seg_softmax_topk_kernel<<<blocks, 64 * SM_WAVES, SM_WAVES * C * sizeof(float), s>>>(
        logits, probs, top_idx, top_prob, seg_off, nseg, B, C);
}

}  // namespace clipvit
