// The classifier head, all fp32 (a 1e-3-relative logit bar leaves no room for 16-bit here):
//   f      = ln_post(x[:, 0, :]) @ proj                    [3p] VisionTransformer.forward tail
//   f_hat  = f / ||f||                                      main.py:205, main.py:445, main.py:504
//   logits = 100 * f_hat @ T^T                              main.py:208, main.py:456, main.py:506
//   probs  = softmax(logits) inside each label segment      (detector 40 | styles | ... )
//   top-k  = topk(min(5, n)) per segment                    main.py:211, main.py:457, main.py:507
// T rows are the cached, already L2-normalised text features (main.py:179-182, 296-311); the
// library keeps them transposed (Tt [E][Cpad]) so the logit loop reads them coalesced.
#include "common.h"

namespace clipvit {

constexpr int HEAD_ROWS = 16;  // images per workgroup

// grid (ceil(B/16), E/64), 256 threads.  LN of 16 CLS rows into LDS, then each thread
// accumulates 4 images x 1 output column over D.
__global__ __launch_bounds__(256) void cls_ln_proj_kernel(const float* __restrict__ x,
                                                          const float* __restrict__ gm,
                                                          const float* __restrict__ bt,
                                                          const float* __restrict__ proj,
                                                          float* __restrict__ f, int B, int N,
                                                          int D, int E) {
    extern __shared__ __attribute__((aligned(16))) float ys[];  // [16][D]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b0 = blockIdx.x * HEAD_ROWS;
    for (int i = wave; i < HEAD_ROWS; i += 4) {
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
    __syncthreads();
    const int e = blockIdx.y * 64 + lane;
    const int ib = wave * 4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int d = 0; d < D; ++d) {
        const float p = proj[(size_t)d * E + e];
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) acc[ii] += ys[(ib + ii) * D + d] * p;
    }
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
        const int b = b0 + ib + ii;
        if (b < B) f[(size_t)b * E + e] = acc[ii];
    }
}

// grid (ceil(B/16), Cpad/64), 256 threads.
__global__ __launch_bounds__(256) void logits_kernel(const float* __restrict__ f,
                                                     const float* __restrict__ Tt,
                                                     float* __restrict__ emb_norm,
                                                     float* __restrict__ logits, int B, int E,
                                                     int C, int Cpad) {
    extern __shared__ __attribute__((aligned(16))) float fs[];  // [16][E]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b0 = blockIdx.x * HEAD_ROWS;
    for (int i = wave; i < HEAD_ROWS; i += 4) {
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
    __syncthreads();
    const int c = blockIdx.y * 64 + lane;
    const int ib = wave * 4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int e = 0; e < E; ++e) {
        const float t = Tt[(size_t)e * Cpad + c];
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) acc[ii] += fs[(ib + ii) * E + e] * t;
    }
    if (c < C) {
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
            const int b = b0 + ib + ii;
            if (b < B) logits[(size_t)b * C + c] = 100.0f * acc[ii];
        }
    }
}

// grid B, one wave per image: per segment softmax and top-min(5, n) (ties -> lower index).
__global__ __launch_bounds__(64) void seg_softmax_topk_kernel(const float* __restrict__ logits,
                                                              float* __restrict__ probs,
                                                              int* __restrict__ top_idx,
                                                              float* __restrict__ top_prob,
                                                              const int* __restrict__ seg_off,
                                                              int nseg, int C) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const float* lr = logits + (size_t)b * C;
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
    dim3 grid((B + HEAD_ROWS - 1) / HEAD_ROWS, E / 64), block(256);
    cls_ln_proj_kernel<<<grid, block, HEAD_ROWS * D * sizeof(float), s>>>(x, g, b, proj, f, B, N,
                                                                          D, E);
}

void launch_logits(hipStream_t s, const float* f, const float* Tt, float* emb_norm, float* logits,
                   int B, int E, int C, int Cpad) {
    dim3 grid((B + HEAD_ROWS - 1) / HEAD_ROWS, Cpad / 64), block(256);
    logits_kernel<<<grid, block, HEAD_ROWS * E * sizeof(float), s>>>(f, Tt, emb_norm, logits, B, E,
                                                                     C, Cpad);
}

void launch_seg_softmax_topk(hipStream_t s, const float* logits, float* probs, int* top_idx,
                             float* top_prob, const int* seg_off, int nseg, int B, int C) {
    seg_softmax_topk_kernel<<<B, 64, 0, s>>>(logits, probs, top_idx, top_prob, seg_off, nseg, C);
}

}  // namespace clipvit
