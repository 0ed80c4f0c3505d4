// GPU preprocessing: CLIP's _transform(n_px) on decoded RGB images.
//
//   Resize(n_px, BICUBIC) -> CenterCrop(n_px) -> ToTensor -> Normalize(mean, std)      [3p]
// as applied at main.py:201, main.py:438 and main.py:489 to PIL images that load_image
// already converted to RGB (main.py:119-128). torchvision hands a PIL image to PIL's own
// Image.resize, so the resampling to match is Pillow's 8-bit two-pass convolution
// (libImaging/Resample.c, Pillow 12.2 in this image): per axis, for output index i,
//   center = (i + 0.5) * scale, support = 2 * max(scale, 1),
//   taps [xmin, xmin + xmax) with xmin = (int)(center - support + 0.5) (>= 0),
//   xmax = min((int)(center + support + 0.5), in) - xmin,
//   w_j = bicubic_a=-0.5((xmin + j - center + 0.5) / max(scale, 1)), normalised to sum 1,
//   then fixed point: k_j = (int)(w_j * 2^22 +- 0.5);
// horizontal pass first (rows the vertical pass needs), uint8 intermediate, then vertical;
// each output = clip8((2^21 + sum_j v_j * k_j) >> 22). An axis whose size does not change is
// an exact copy (Pillow skips the pass; an identity plan reproduces it).
//
// The plans (bounds + fixed-point weights) are computed on the host in double precision with
// Pillow's operation order (no FMA contraction), so every output byte is bit-identical to
// PIL; ToTensor/Normalize are the same fp32 IEEE ops torchvision / preprocess.py apply
// ((u8 / 255 - mean) / std). Only the n_px x n_px centre crop is computed.
//
// Device work per call: one horizontal kernel over (crop columns x source rows the crop
// needs) and one vertical kernel over the crop, both one thread per pixel (3 channels),
// writing [B, 3, n_px, n_px] fp32 / bf16 / fp16 for clipvit_encode_image / clipvit_classify.
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "clipvit.h"
#include "common.h"

namespace clipvit {

extern thread_local std::string g_err;

namespace {

constexpr int PRECISION_BITS = 32 - 8 - 2;

#pragma clang fp contract(off)
double bicubic_filter(double x) {  // Pillow's bicubic, a = -0.5, support 2
    const double a = -0.5;
    if (x < 0.0) x = -x;
    if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
    if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
    return 0.0;
}

struct Plan {
    int ksize = 1;
    std::vector<int> bounds;   // [out][2] = xmin, xmax (tap count)
    std::vector<int32_t> kk;   // [out][ksize] fixed point, PRECISION_BITS fraction bits
};

// Pillow precompute_coeffs + normalize_coeffs_8bpc for box (0, in); identity when out == in.
Plan make_plan(int in, int out) {
    Plan p;
    p.bounds.resize((size_t)out * 2);
    if (in == out) {
        p.ksize = 1;
        p.kk.assign((size_t)out, 1 << PRECISION_BITS);
        for (int i = 0; i < out; ++i) { p.bounds[2 * i] = i; p.bounds[2 * i + 1] = 1; }
        return p;
    }
    const double in0 = 0.0, in1 = (double)in;
    double filterscale, scale;
    filterscale = scale = (double)(in1 - in0) / out;
    if (filterscale < 1.0) filterscale = 1.0;
    const double support = 2.0 * filterscale;
    const int ksize = (int)std::ceil(support) * 2 + 1;
    p.ksize = ksize;
    std::vector<double> kd((size_t)out * ksize, 0.0);
    for (int xx = 0; xx < out; ++xx) {
        const double center = in0 + (xx + 0.5) * scale;
        double ww = 0.0;
        const double ss = 1.0 / filterscale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in) xmax = in;
        xmax -= xmin;
        double* k = &kd[(size_t)xx * ksize];
        for (int x = 0; x < xmax; ++x) {
            const double w = bicubic_filter((x + xmin - center + 0.5) * ss);
            k[x] = w;
            ww += w;
        }
        for (int x = 0; x < xmax; ++x)
            if (ww != 0.0) k[x] /= ww;
        p.bounds[2 * xx] = xmin;
        p.bounds[2 * xx + 1] = xmax;
    }
    p.kk.resize(kd.size());
    for (size_t x = 0; x < kd.size(); ++x)
        p.kk[x] = kd[x] < 0 ? (int32_t)(-0.5 + kd[x] * (1 << PRECISION_BITS))
                            : (int32_t)(0.5 + kd[x] * (1 << PRECISION_BITS));
    return p;
}
#pragma clang fp contract(on)

// torchvision Resize(int) on a PIL image: short side -> n, long side int(n * long / short)
void resize_size(int w, int h, int n, int& nw, int& nh) {
    if (w <= h) { nw = n; nh = (int)((long long)n * h / w); }
    else { nw = (int)((long long)n * w / h); nh = n; }
}
// CenterCrop offset: int(round((size - n) / 2.0)) with Python's round-half-to-even
int crop_offset(int size, int n) {
    return (int)std::nearbyint((size - n) / 2.0);  // default FE_TONEAREST = ties to even
}

struct ImgDesc {
    long long src;    // byte offset of the image (HWC uint8 RGB) in the input buffer
    long long inter;  // byte offset of its intermediate [R][n][3] uint8 block
    int W, H;
    int rlo, R;       // first source row the crop needs, number of rows
    int left, top;    // crop origin in the resized image
    int ksh, ksv;     // taps per output column / row
    int bh, kh, bv, kv;  // int32 offsets of the plans in the plan buffer
};

__device__ __forceinline__ unsigned char clip8(int in) {
    if (in >= (1 << PRECISION_BITS << 8)) return 255;
    if (in <= 0) return 0;
    return (unsigned char)(in >> PRECISION_BITS);
}

// intermediate[b][r][c] = horizontal resample of source row rlo + r at output column left + c
__global__ __launch_bounds__(256) void resample_h_kernel(const unsigned char* __restrict__ rgb,
                                                         const ImgDesc* __restrict__ descs,
                                                         const int32_t* __restrict__ plans,
                                                         unsigned char* __restrict__ inter, int n) {
    const ImgDesc d = descs[blockIdx.y];
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long long)d.R * n) return;
    const int r = (int)(t / n), c = (int)(t % n);
    const int xx = d.left + c;
    const int xmin = plans[d.bh + 2 * xx], xmax = plans[d.bh + 2 * xx + 1];
    const int32_t* k = plans + d.kh + (size_t)xx * d.ksh;
    const unsigned char* s = rgb + d.src + ((size_t)(d.rlo + r) * d.W + xmin) * 3;
    int s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < xmax; ++x) {
        const int w = k[x];
        s0 += (int)s[3 * x] * w;
        s1 += (int)s[3 * x + 1] * w;
        s2 += (int)s[3 * x + 2] * w;
    }
    unsigned char* o = inter + d.inter + (size_t)t * 3;
    o[0] = clip8(s0);
    o[1] = clip8(s1);
    o[2] = clip8(s2);
}

// Same output, one workgroup per (source row, image): the row's needed byte span is staged in
// LDS by coalesced loads, then each thread computes output columns from LDS (the per-thread
// version issues 3 scattered byte loads per tap). Dynamic LDS = span bytes (<= 48 KiB).
__global__ __launch_bounds__(256) void resample_h_lds_kernel(const unsigned char* __restrict__ rgb,
                                                             const ImgDesc* __restrict__ descs,
                                                             const int32_t* __restrict__ plans,
                                                             unsigned char* __restrict__ inter, int n) {
    extern __shared__ unsigned char row[];
    const ImgDesc d = descs[blockIdx.y];
    const int r = blockIdx.x;
    if (r >= d.R) return;
    const int x0 = plans[d.bh + 2 * d.left];
    const int lc = d.left + n - 1;
    const int span = (plans[d.bh + 2 * lc] + plans[d.bh + 2 * lc + 1] - x0) * 3;
    const unsigned char* src = rgb + d.src + ((size_t)(d.rlo + r) * d.W + x0) * 3;
    for (int i = threadIdx.x; i < span; i += blockDim.x) row[i] = src[i];
    __syncthreads();
    unsigned char* o = inter + d.inter + (size_t)r * n * 3;
    for (int c = threadIdx.x; c < n; c += blockDim.x) {
        const int xx = d.left + c;
        const int xmin = plans[d.bh + 2 * xx], xmax = plans[d.bh + 2 * xx + 1];
        const int32_t* k = plans + d.kh + (size_t)xx * d.ksh;
        const unsigned char* sp = row + (xmin - x0) * 3;
        int s0 = 1 << (PRECISION_BITS - 1), s1 = s0, s2 = s0;
        for (int x = 0; x < xmax; ++x) {
            const int w = k[x];
            s0 += (int)sp[3 * x] * w;
            s1 += (int)sp[3 * x + 1] * w;
            s2 += (int)sp[3 * x + 2] * w;
        }
        o[3 * c] = clip8(s0);
        o[3 * c + 1] = clip8(s1);
        o[3 * c + 2] = clip8(s2);
    }
}

template <int OUT>  // 0 fp32, 1 bf16, 2 fp16
__global__ __launch_bounds__(256) void resample_v_kernel(const ImgDesc* __restrict__ descs,
                                                         const int32_t* __restrict__ plans,
                                                         const unsigned char* __restrict__ inter,
                                                         void* __restrict__ out, int n) {
    const int b = blockIdx.y;
    const ImgDesc d = descs[b];
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * n) return;
    const int y = t / n, c = t % n;
    const int yy = d.top + y;
    const int ymin = plans[d.bv + 2 * yy] - d.rlo, ymax = plans[d.bv + 2 * yy + 1];
    const int32_t* k = plans + d.kv + (size_t)yy * d.ksv;
    const unsigned char* s = inter + d.inter + ((size_t)ymin * n + c) * 3;
    int acc[3] = {1 << (PRECISION_BITS - 1), 1 << (PRECISION_BITS - 1), 1 << (PRECISION_BITS - 1)};
    for (int j = 0; j < ymax; ++j) {
        const int w = k[j];
        const unsigned char* p = s + (size_t)j * n * 3;
        acc[0] += (int)p[0] * w;
        acc[1] += (int)p[1] * w;
        acc[2] += (int)p[2] * w;
    }
    const float mean[3] = {0.48145466f, 0.4578275f, 0.40821073f};
    const float stdv[3] = {0.26862954f, 0.26130258f, 0.27577711f};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const float v = ((float)clip8(acc[ch]) / 255.0f - mean[ch]) / stdv[ch];
        const size_t o = (((size_t)b * 3 + ch) * n + y) * n + c;
        if constexpr (OUT == 0) ((float*)out)[o] = v;
        else if constexpr (OUT == 1) ((u16*)out)[o] = BF16::from_f32(v);
        else ((u16*)out)[o] = F16::from_f32(v);
    }
}

}  // namespace
}  // namespace clipvit

using namespace clipvit;

#define PP_FAIL(code, msg)   \
    do {                     \
        g_err = (msg);       \
        return (code);       \
    } while (0)

extern "C" {

int clipvit_resample_plan(int in_size, int out_size, int* ksize, int* bounds, int32_t* kk, int kk_cap) {
    g_err.clear();
    if (in_size <= 0 || out_size <= 0 || !ksize || !bounds || !kk) PP_FAIL(CLIPVIT_E_INVALID, "bad argument");
    const Plan p = make_plan(in_size, out_size);
    *ksize = p.ksize;
    if ((size_t)kk_cap < p.kk.size()) PP_FAIL(CLIPVIT_E_INVALID, "kk buffer too small");
    for (size_t i = 0; i < p.bounds.size(); ++i) bounds[i] = p.bounds[i];
    for (size_t i = 0; i < p.kk.size(); ++i) kk[i] = p.kk[i];
    return 0;
}

int clipvit_preprocess(void* stream, const unsigned char* rgb_dev, const clipvit_image* images, int B,
                       int n_px, int out_dtype, void* out_dev) {
    g_err.clear();
    if (!rgb_dev || !images || !out_dev || B <= 0 || n_px <= 0) PP_FAIL(CLIPVIT_E_INVALID, "bad argument");
    if (out_dtype < 0 || out_dtype > 2) PP_FAIL(CLIPVIT_E_INVALID, "out_dtype must be F32, BF16 or F16");
    hipStream_t s = (hipStream_t)stream;
    std::vector<ImgDesc> descs((size_t)B);
    std::vector<int32_t> plans;
    long long inter_bytes = 0;
    int maxR = 0, maxSpan = 0;
    // plans depend only on (source size, resized size): one copy per distinct axis pair (a
    // batch of same-size photos uploads two plans, not 2 B)
    struct PlanRef { int b, k, ks, first; };
    std::map<std::pair<int, int>, PlanRef> cache;
    auto plan_of = [&](int in, int out) -> PlanRef {
        auto it = cache.find({in, out});
        if (it != cache.end()) return it->second;
        const Plan p = make_plan(in, out);
        PlanRef r{(int)plans.size(), 0, p.ksize, p.bounds[0]};
        plans.insert(plans.end(), p.bounds.begin(), p.bounds.end());
        r.k = (int)plans.size();
        plans.insert(plans.end(), p.kk.begin(), p.kk.end());
        cache.emplace(std::make_pair(in, out), r);
        return r;
    };
    for (int b = 0; b < B; ++b) {
        const clipvit_image& im = images[b];
        if (im.width <= 0 || im.height <= 0 || im.offset < 0)
            PP_FAIL(CLIPVIT_E_INVALID, "image " + std::to_string(b) + ": bad size/offset");
        int nw, nh;
        resize_size(im.width, im.height, n_px, nw, nh);
        if (nw < n_px || nh < n_px) PP_FAIL(CLIPVIT_E_INVALID, "resized image smaller than the crop");
        const PlanRef ph = plan_of(im.width, nw), pv = plan_of(im.height, nh);
        ImgDesc& d = descs[b];
        d.src = im.offset;
        d.W = im.width;
        d.H = im.height;
        d.left = crop_offset(nw, n_px);
        d.top = crop_offset(nh, n_px);
        d.ksh = ph.ks;
        d.ksv = pv.ks;
        d.rlo = plans[pv.b + 2 * d.top];
        const int last = d.top + n_px - 1;
        d.R = plans[pv.b + 2 * last] + plans[pv.b + 2 * last + 1] - d.rlo;
        d.inter = inter_bytes;
        inter_bytes += (long long)d.R * n_px * 3;
        maxR = std::max(maxR, d.R);
        {
            const int lc = d.left + n_px - 1;
            const int span = (plans[ph.b + 2 * lc] + plans[ph.b + 2 * lc + 1] - plans[ph.b + 2 * d.left]) * 3;
            maxSpan = std::max(maxSpan, span);
        }
        d.bh = ph.b;
        d.kh = ph.k;
        d.bv = pv.b;
        d.kv = pv.k;
    }
    // one device block: descs | plans | intermediate
    const size_t dbytes = descs.size() * sizeof(ImgDesc), pbytes = plans.size() * sizeof(int32_t);
    const size_t poff = (dbytes + 255) / 256 * 256, ioff = (poff + pbytes + 255) / 256 * 256;
    void* blk = nullptr;
    hipError_t e = hipMallocAsync(&blk, ioff + (size_t)inter_bytes, s);
    if (e != hipSuccess) PP_FAIL(CLIPVIT_E_NOMEM, std::string("preprocess workspace: ") + hipGetErrorString(e));
    // the staging copy lives until the stream has consumed it (freed by a host callback)
    auto* host = new std::vector<unsigned char>(poff + pbytes);
    std::memcpy(host->data(), descs.data(), dbytes);
    std::memcpy(host->data() + poff, plans.data(), pbytes);
    e = hipMemcpyAsync(blk, host->data(), host->size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = hipLaunchHostFunc(s, [](void* p) { delete (std::vector<unsigned char>*)p; }, host);
    else
        delete host;
    const ImgDesc* ddesc = (const ImgDesc*)blk;
    const int32_t* dplans = (const int32_t*)((char*)blk + poff);
    unsigned char* dinter = (unsigned char*)blk + ioff;
    if (e == hipSuccess) {
        if (maxSpan <= 48 * 1024) {
            resample_h_lds_kernel<<<dim3((unsigned)maxR, (unsigned)B), 256, maxSpan, s>>>(rgb_dev, ddesc, dplans,
                                                                                     dinter, n_px);
        } else {
            dim3 gh((unsigned)(((long long)maxR * n_px + 255) / 256), (unsigned)B);
            resample_h_kernel<<<gh, 256, 0, s>>>(rgb_dev, ddesc, dplans, dinter, n_px);
        }
        dim3 gv((unsigned)((n_px * n_px + 255) / 256), (unsigned)B);
        if (out_dtype == CLIPVIT_F32) resample_v_kernel<0><<<gv, 256, 0, s>>>(ddesc, dplans, dinter, out_dev, n_px);
        else if (out_dtype == CLIPVIT_BF16) resample_v_kernel<1><<<gv, 256, 0, s>>>(ddesc, dplans, dinter, out_dev, n_px);
        else resample_v_kernel<2><<<gv, 256, 0, s>>>(ddesc, dplans, dinter, out_dev, n_px);
        e = hipGetLastError();
    }
    const hipError_t e2 = hipFreeAsync(blk, s);
    if (e != hipSuccess) PP_FAIL(CLIPVIT_E_HIP, std::string("preprocess: ") + hipGetErrorString(e));
    if (e2 != hipSuccess) PP_FAIL(CLIPVIT_E_HIP, std::string("preprocess free: ") + hipGetErrorString(e2));
    return 0;
}

}  // extern "C"
