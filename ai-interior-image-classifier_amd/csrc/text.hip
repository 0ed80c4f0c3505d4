// Text tower of CLIP on gfx950: model.encode_text(clip.tokenize(p))
// as the reference runs it once per prompt set — InteriorImageDetector (main.py:179-182, the
// 40 detector prompts, base model) and CachedInteriorAnalyzer._precompute_text_features_
// optimized (main.py:296-311, 397 analyzer prompts, LoRA model). The shipped checkpoints'
// adapters live exactly here (text mlp.c_fc / mlp.c_proj, r = 4), so regenerating the label
// matrix T with LoRA needs this tower; the result feeds clipvit_set_text_features.
//
//   x = token_embedding[ids] + positional_embedding          (text_embed_ln_kernel, + ln_1)
//   12x [ QKV GEMM -> causal attention -> out GEMM (+x) -> LN -> c_fc GEMM (QuickGELU)
//         -> c_proj GEMM (+x) -> LN ]                          (the vision tower's kernels)
//   f = ln_final(x[b, argmax(ids[b])]) @ text_projection       (eot_gather + cls_ln_proj)
//   optionally f /= ||f||                                      (main.py:182, main.py:309)
//
// Same fixed kernel sequence, packed 16-bit MFMA operands and fp32 residual stream as the
// vision path (clipvit.hip); residual adds use the fp32 read-modify-write epilogue (the text
// tower runs once per label set, so the simplest exact form is used). Token ids are clamped to
// [0, vocab) on the device; the Python layer rejects out-of-range ids before the call.
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "clipvit.h"
#include "common.h"

namespace clipvit {

extern thread_local std::string g_err;

namespace {

// x[row] = tok[clamp(id)] + pos[t];  h[row] = ln(x[row])   (one wave per token row)
template <typename T, int V>
__global__ __launch_bounds__(256) void text_embed_ln_kernel(const int* __restrict__ ids,
                                                            const float* __restrict__ tok,
                                                            const float* __restrict__ pos,
                                                            const float* __restrict__ g,
                                                            const float* __restrict__ b,
                                                            float* __restrict__ x, u16* __restrict__ h,
                                                            int rows, int ctx, int vocab) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= rows) return;
    constexpr int D = 256 * V;
    int id = ids[row];
    id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
    const int t = row % ctx;
    float4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const int c = (lane + 64 * i) * 4;
        const float4 a = *(const float4*)(tok + (size_t)id * D + c);
        const float4 p = *(const float4*)(pos + (size_t)t * D + c);
        v[i] = make_float4(a.x + p.x, a.y + p.y, a.z + p.z, a.w + p.w);
        *(float4*)(x + (size_t)row * D + c) = v[i];
    }
    ln_row<V>(v, g, b, lane, (float)D);
    store_row16<T, V>(h + (size_t)row * D, v, lane);
}

// out[b] = x[b * ctx + argmax_t ids[b, t]] (first maximum, torch.argmax) — one wave per text
__global__ __launch_bounds__(64) void eot_gather_kernel(const int* __restrict__ ids,
                                                        const float* __restrict__ x,
                                                        float* __restrict__ out, int ctx, int D) {
    const int b = blockIdx.x, lane = threadIdx.x;
    int best = -2147483647 - 1, at = 0;
    for (int t = lane; t < ctx; t += 64) {
        const int v = ids[(size_t)b * ctx + t];
        if (v > best) { best = v; at = t; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int ob = __shfl_xor(best, o, 64), oa = __shfl_xor(at, o, 64);
        if (ob > best || (ob == best && oa < at)) { best = ob; at = oa; }
    }
    const float* src = x + ((size_t)b * ctx + at) * D;
    for (int c = lane * 4; c < D; c += 256)
        *(float4*)(out + (size_t)b * D + c) = *(const float4*)(src + c);
}

// f[b] /= ||f[b]||_2   (one wave per row)
__global__ __launch_bounds__(64) void l2_normalize_kernel(float* __restrict__ f, int E) {
    float* r = f + (size_t)blockIdx.x * E;
    float s = 0.f;
    for (int c = threadIdx.x; c < E; c += 64) s += r[c] * r[c];
    const float inv = 1.0f / sqrtf(wave_sum(s));
    for (int c = threadIdx.x; c < E; c += 64) r[c] *= inv;
}

struct TextLayer {
    void *wqkv = nullptr, *wout = nullptr, *wfc = nullptr, *wproj = nullptr;
    const float *bqkv, *bout, *bfc, *bproj, *ln1g, *ln1b, *ln2g, *ln2b;
};

std::string TL(int i, const char* leaf) {
    return "transformer.resblocks." + std::to_string(i) + "." + leaf;
}

}  // namespace
}  // namespace clipvit

using namespace clipvit;

struct clipvit_text_handle {
    clipvit_text_config cfg{};
    int device = 0, dt = CLIPVIT_F16;
    std::unordered_map<std::string, float*> master;
    std::unordered_map<std::string, std::vector<int64_t>> shapes;
    std::vector<TextLayer> layers;
    bool loaded = false;
    float* scratch = nullptr;  // [4D * D] fp32: LoRA merge target
    // workspace for max_batch texts (one call at a time; ordered by `done`)
    std::mutex mu;
    float *x = nullptr, *eot = nullptr, *f = nullptr;
    void *h = nullptr, *qkv = nullptr, *u = nullptr;
    hipEvent_t done = nullptr;
    // GEMM tiles (qkv, out, fc, proj) and the fp16 residual
    // scheme of the vision tower (16-bit branch outputs + add_layernorm, deferred x store).
    // Measured on the 437 label prompts (M = 33,649): fc on 128x128 (v13) 4.84 ms per call
    // against 4.88-4.90 on 256x256 (v8: 1,056 tiles = 4.1 rounds); qkv 240x256 / 160x128 no
    // better than 256x256; resid16 4.89 against 5.00 ms with the fp32 epilogue adds
    // (fc: the 128x128 tile 81 since the direct-store 128x128 tile 13 was retired in r04)
    int var[4] = {80, 82, 81, 82};
    bool resid16 = false;
};

#define TFAIL(code, msg) \
    do {                 \
        g_err = (msg);   \
        return (code);   \
    } while (0)
#define THIP(x)                                                                  \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            g_err = std::string(#x) + " failed: " + hipGetErrorString(e_);      \
            return CLIPVIT_E_HIP;                                                \
        }                                                                        \
    } while (0)

static void text_expected(const clipvit_text_handle* h,
                          std::vector<std::pair<std::string, std::vector<int64_t>>>& out) {
    const int64_t D = h->cfg.width;
    out.push_back({"token_embedding.weight", {h->cfg.vocab, D}});
    out.push_back({"positional_embedding", {h->cfg.context, D}});
    for (int i = 0; i < h->cfg.layers; ++i) {
        out.push_back({TL(i, "ln_1.weight"), {D}});
        out.push_back({TL(i, "ln_1.bias"), {D}});
        out.push_back({TL(i, "attn.in_proj_weight"), {3 * D, D}});
        out.push_back({TL(i, "attn.in_proj_bias"), {3 * D}});
        out.push_back({TL(i, "attn.out_proj.weight"), {D, D}});
        out.push_back({TL(i, "attn.out_proj.bias"), {D}});
        out.push_back({TL(i, "ln_2.weight"), {D}});
        out.push_back({TL(i, "ln_2.bias"), {D}});
        out.push_back({TL(i, "mlp.c_fc.weight"), {4 * D, D}});
        out.push_back({TL(i, "mlp.c_fc.bias"), {4 * D}});
        out.push_back({TL(i, "mlp.c_proj.weight"), {D, 4 * D}});
        out.push_back({TL(i, "mlp.c_proj.bias"), {D}});
    }
    out.push_back({"ln_final.weight", {D}});
    out.push_back({"ln_final.bias", {D}});
    out.push_back({"text_projection", {D, h->cfg.embed_dim}});
}

static void text_pack(clipvit_text_handle* h, const std::string& name, void* dst, const float* src) {
    const auto& sh = h->shapes[name];
    launch_pack_weight(nullptr, h->dt, src ? src : h->master[name], dst, (int)sh[0], (int)sh[1], (int)sh[1]);
}

// variant: the vision roles' pipelined tiles (h->var; N = 512 roles with the 4x2 XCD partition),
// falling back to the shape-based choice
static int text_gemm(hipStream_t s, clipvit_text_handle* h, int epi, const void* A, const void* W,
                     const float* bias, void* C, int M, int N, int K, int variant) {
    GemmArgs a{};
    a.A = A; a.W = W; a.bias = bias; a.C = C;
    a.M = M; a.N = N; a.K = K; a.ldc = N;
    a.xcd_n = 2;
    if (launch_gemm(s, h->dt, epi, a, variant) != 0 && launch_gemm(s, h->dt, epi, a, 0) != 0)
        TFAIL(CLIPVIT_E_INVALID, "text gemm: unsupported shape M=" + std::to_string(M) +
                                     " N=" + std::to_string(N) + " K=" + std::to_string(K));
    return 0;
}

template <typename T>
static void launch_text_embed(hipStream_t s, clipvit_text_handle* h, const int* ids, int rows) {
    const float* tok = h->master["token_embedding.weight"];
    const float* pos = h->master["positional_embedding"];
    const TextLayer& l0 = h->layers[0];
    const int D = h->cfg.width;
    dim3 grid((rows + 3) / 4), block(256);
    switch (D / 256) {
        case 2: text_embed_ln_kernel<T, 2><<<grid, block, 0, s>>>(ids, tok, pos, l0.ln1g, l0.ln1b, h->x, (u16*)h->h, rows, h->cfg.context, h->cfg.vocab); break;
        case 3: text_embed_ln_kernel<T, 3><<<grid, block, 0, s>>>(ids, tok, pos, l0.ln1g, l0.ln1b, h->x, (u16*)h->h, rows, h->cfg.context, h->cfg.vocab); break;
        case 4: text_embed_ln_kernel<T, 4><<<grid, block, 0, s>>>(ids, tok, pos, l0.ln1g, l0.ln1b, h->x, (u16*)h->h, rows, h->cfg.context, h->cfg.vocab); break;
        default: break;
    }
}

extern "C" {

int clipvit_text_create(const clipvit_text_config* cfg, int device, clipvit_text_handle** out) {
    g_err.clear();
    if (!cfg || !out) TFAIL(CLIPVIT_E_INVALID, "null argument");
    const clipvit_text_config& c = *cfg;
    if (c.width % 256 || c.width < 512 || c.width > 1024)
        TFAIL(CLIPVIT_E_INVALID, "text width must be a multiple of 256 in [512, 1024]");
    if (c.heads * 64 != c.width) TFAIL(CLIPVIT_E_INVALID, "heads * 64 must equal width");
    if (c.embed_dim % 64 || c.embed_dim <= 0 || c.embed_dim > 1280)
        TFAIL(CLIPVIT_E_INVALID, "embed_dim must be a multiple of 64 in [64, 1280]");
    if (c.layers <= 0 || c.context <= 0 || c.context > 1024 || c.vocab <= 0 || c.max_batch <= 0)
        TFAIL(CLIPVIT_E_INVALID, "layers/context/vocab/max_batch out of range");
    if (c.compute_dtype != CLIPVIT_BF16 && c.compute_dtype != CLIPVIT_F16)
        TFAIL(CLIPVIT_E_INVALID, "text compute_dtype must be BF16 or F16");
    int ndev = 0;
    THIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) TFAIL(CLIPVIT_E_INVALID, "bad device index");
    auto* h = new clipvit_text_handle();
    h->cfg = c;
    h->device = device;
    h->dt = c.compute_dtype;
    h->resid16 = true;  // both 16-bit types, as the vision tower
    *out = h;
    return 0;
}

int clipvit_text_load_weights(clipvit_text_handle* h, const clipvit_tensor* tensors, size_t n) {
    g_err.clear();
    if (!h || (!tensors && n)) TFAIL(CLIPVIT_E_INVALID, "null argument");
    THIP(hipSetDevice(h->device));
    std::unordered_map<std::string, const clipvit_tensor*> byname;
    for (size_t i = 0; i < n; ++i)
        if (tensors[i].name) byname[tensors[i].name] = &tensors[i];
    std::vector<std::pair<std::string, std::vector<int64_t>>> exp;
    text_expected(h, exp);
    for (auto& e : exp) {
        auto it = byname.find(e.first);
        if (it == byname.end()) TFAIL(CLIPVIT_E_INVALID, "missing tensor " + e.first);
        const clipvit_tensor* t = it->second;
        bool ok = t->ndim == (int)e.second.size() && t->data;
        for (int d = 0; ok && d < t->ndim; ++d) ok = t->shape[d] == e.second[d];
        if (!ok) TFAIL(CLIPVIT_E_INVALID, "bad shape/data for " + e.first);
    }
    for (auto& e : exp) {
        size_t cnt = 1;
        for (auto d : e.second) cnt *= (size_t)d;
        float*& dst = h->master[e.first];
        if (!dst) THIP(hipMalloc(&dst, cnt * sizeof(float)));
        THIP(hipMemcpy(dst, byname[e.first]->data, cnt * sizeof(float), hipMemcpyHostToDevice));
        h->shapes[e.first] = e.second;
    }
    const size_t D = h->cfg.width;
    h->layers.resize(h->cfg.layers);
    for (int i = 0; i < h->cfg.layers; ++i) {
        TextLayer& ly = h->layers[i];
        if (!ly.wqkv) THIP(hipMalloc(&ly.wqkv, 3 * D * D * 2));
        if (!ly.wout) THIP(hipMalloc(&ly.wout, D * D * 2));
        if (!ly.wfc) THIP(hipMalloc(&ly.wfc, 4 * D * D * 2));
        if (!ly.wproj) THIP(hipMalloc(&ly.wproj, 4 * D * D * 2));
        ly.bqkv = h->master[TL(i, "attn.in_proj_bias")];
        ly.bout = h->master[TL(i, "attn.out_proj.bias")];
        ly.bfc = h->master[TL(i, "mlp.c_fc.bias")];
        ly.bproj = h->master[TL(i, "mlp.c_proj.bias")];
        ly.ln1g = h->master[TL(i, "ln_1.weight")];
        ly.ln1b = h->master[TL(i, "ln_1.bias")];
        ly.ln2g = h->master[TL(i, "ln_2.weight")];
        ly.ln2b = h->master[TL(i, "ln_2.bias")];
        text_pack(h, TL(i, "attn.in_proj_weight"), ly.wqkv, nullptr);
        text_pack(h, TL(i, "attn.out_proj.weight"), ly.wout, nullptr);
        text_pack(h, TL(i, "mlp.c_fc.weight"), ly.wfc, nullptr);
        text_pack(h, TL(i, "mlp.c_proj.weight"), ly.wproj, nullptr);
    }
    if (!h->scratch) THIP(hipMalloc(&h->scratch, 4 * D * D * sizeof(float)));
    if (!h->x) {
        const size_t rows = (size_t)h->cfg.max_batch * h->cfg.context;
        THIP(hipMalloc(&h->x, rows * D * sizeof(float)));
        THIP(hipMalloc(&h->h, rows * D * 2));
        THIP(hipMalloc(&h->qkv, rows * 3 * D * 2));
        THIP(hipMalloc(&h->u, rows * 4 * D * 2));
        THIP(hipMalloc(&h->eot, (size_t)h->cfg.max_batch * D * sizeof(float)));
        THIP(hipEventCreateWithFlags(&h->done, hipEventDisableTiming));
    }
    THIP(hipGetLastError());
    THIP(hipDeviceSynchronize());
    h->loaded = true;
    return 0;
}

int clipvit_text_load_lora(clipvit_text_handle* h, const clipvit_lora* items, size_t n) {
    g_err.clear();
    if (!h || (!items && n)) TFAIL(CLIPVIT_E_INVALID, "null argument");
    if (!h->loaded) TFAIL(CLIPVIT_E_STATE, "weights not loaded");
    THIP(hipSetDevice(h->device));
    std::unordered_map<std::string, void*> dst;
    for (int i = 0; i < h->cfg.layers; ++i) {
        dst[TL(i, "attn.in_proj_weight")] = h->layers[i].wqkv;
        dst[TL(i, "attn.out_proj.weight")] = h->layers[i].wout;
        dst[TL(i, "mlp.c_fc.weight")] = h->layers[i].wfc;
        dst[TL(i, "mlp.c_proj.weight")] = h->layers[i].wproj;
    }
    for (size_t k = 0; k < n; ++k) {
        const clipvit_lora& it = items[k];
        if (!it.target || !dst.count(it.target))
            TFAIL(CLIPVIT_E_INVALID, std::string("unknown text LoRA target ") + (it.target ? it.target : "(null)"));
        const auto& sh = h->shapes[it.target];
        if (sh[0] != it.out_features || sh[1] != it.in_features || it.rank <= 0 || !it.A || !it.B)
            TFAIL(CLIPVIT_E_INVALID, std::string("LoRA shape mismatch for ") + it.target);
    }
    std::lock_guard<std::mutex> lk(h->mu);
    THIP(hipDeviceSynchronize());  // no encode may read the packed weights while they change
    for (auto& kv : dst) text_pack(h, kv.first, kv.second, nullptr);  // base weights, then merges
    std::unordered_map<std::string, std::vector<size_t>> groups;
    for (size_t k = 0; k < n; ++k) groups[items[k].target].push_back(k);
    for (auto& gkv : groups) {
        const auto& sh = h->shapes[gkv.first];
        const size_t cnt = (size_t)sh[0] * sh[1];
        THIP(hipMemcpy(h->scratch, h->master[gkv.first], cnt * sizeof(float), hipMemcpyDeviceToDevice));
        for (size_t k : gkv.second) {
            const clipvit_lora& it = items[k];
            const size_t na = (size_t)it.in_features * it.rank, nb = (size_t)it.rank * it.out_features;
            float* dAB = nullptr;
            THIP(hipMalloc(&dAB, (na + nb) * sizeof(float)));
            hipError_t e = hipMemcpy(dAB, it.A, na * sizeof(float), hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(dAB + na, it.B, nb * sizeof(float), hipMemcpyHostToDevice);
            if (e == hipSuccess) {
                launch_lora_merge(nullptr, h->scratch, dAB, dAB + na, it.in_features, it.out_features,
                                  it.rank, it.scaling);
                e = hipDeviceSynchronize();
            }
            hipFree(dAB);
            THIP(e);
        }
        text_pack(h, gkv.first, dst[gkv.first], h->scratch);
        THIP(hipDeviceSynchronize());
    }
    THIP(hipGetLastError());
    return 0;
}

int clipvit_encode_text(clipvit_text_handle* h, void* stream, const int32_t* tokens_dev, int B,
                        int l2_normalize, float* out_dev) {
    g_err.clear();
    if (!h) TFAIL(CLIPVIT_E_INVALID, "null handle");
    if (!h->loaded) TFAIL(CLIPVIT_E_STATE, "weights not loaded");
    if (!tokens_dev || !out_dev) TFAIL(CLIPVIT_E_INVALID, "null buffer");
    if (B <= 0 || B > h->cfg.max_batch)
        TFAIL(CLIPVIT_E_INVALID, "batch " + std::to_string(B) + " outside [1, max_batch=" +
                                     std::to_string(h->cfg.max_batch) + "]");
    THIP(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    const int D = h->cfg.width, ctx = h->cfg.context, M = B * ctx, E = h->cfg.embed_dim;
    std::lock_guard<std::mutex> lk(h->mu);
    THIP(hipStreamWaitEvent(s, h->done, 0));
    if (h->dt == CLIPVIT_F16) launch_text_embed<F16>(s, h, tokens_dev, M);
    else launch_text_embed<BF16>(s, h, tokens_dev, M);
    int rc = 0;
    // resid16: out_proj / c_proj store their 16-bit branch outputs y, y2 into the qkv buffer (dead
    // once attention has read it) and add_layernorm does the residual adds, x stored once per
    // block ((x + y) + y2, the vision tower's deferred scheme, clipvit.hip forward()); the last
    // block's c_proj adds into x in its epilogue (the EOT gather reads x). resid16 = false:
    // fp32 residual read-modify-write in the GEMM epilogues.
    void* y = h->qkv;
    void* y2 = (u16*)h->qkv + (size_t)M * D;
    const int* v = h->var;
    for (int i = 0; i < h->cfg.layers && !rc; ++i) {
        const TextLayer& ly = h->layers[i];
        const bool last = i + 1 == h->cfg.layers;
        if ((rc = text_gemm(s, h, EPI_STORE, h->h, ly.wqkv, ly.bqkv, h->qkv, M, 3 * D, D, v[0]))) break;
        launch_attention(s, h->dt, h->qkv, h->h, B, ctx, h->cfg.heads, /*causal=*/true);
        if (h->resid16) {
            if ((rc = text_gemm(s, h, EPI_STORE, h->h, ly.wout, ly.bout, y, M, D, D, v[1]))) break;
            if (last) launch_add_layernorm(s, h->dt, h->x, y, h->h, ly.ln2g, ly.ln2b, M, D);
            else launch_add_layernorm_deferred(s, h->dt, h->x, y, nullptr, h->h, ly.ln2g, ly.ln2b, M, D);
        } else {
            if ((rc = text_gemm(s, h, EPI_RESID, h->h, ly.wout, ly.bout, h->x, M, D, D, v[1]))) break;
            launch_layernorm(s, h->dt, h->x, h->h, ly.ln2g, ly.ln2b, M, D);
        }
        if ((rc = text_gemm(s, h, EPI_GELU, h->h, ly.wfc, ly.bfc, h->u, M, 4 * D, D, v[2]))) break;
        if (h->resid16 && !last) {
            if ((rc = text_gemm(s, h, EPI_STORE, h->u, ly.wproj, ly.bproj, y2, M, D, 4 * D, v[3]))) break;
            const TextLayer& nx = h->layers[i + 1];
            launch_add_layernorm_deferred(s, h->dt, h->x, y, y2, h->h, nx.ln1g, nx.ln1b, M, D);
        } else {
            if ((rc = text_gemm(s, h, EPI_RESID, h->u, ly.wproj, ly.bproj, h->x, M, D, 4 * D, v[3]))) break;
            if (!last)
                launch_layernorm(s, h->dt, h->x, h->h, h->layers[i + 1].ln1g, h->layers[i + 1].ln1b, M, D);
        }
    }
    if (!rc) {
        eot_gather_kernel<<<B, 64, 0, s>>>(tokens_dev, h->x, h->eot, ctx, D);
        launch_cls_ln_proj(s, h->eot, h->master["ln_final.weight"], h->master["ln_final.bias"],
                           h->master["text_projection"], out_dev, B, 1, D, E);
        if (l2_normalize) l2_normalize_kernel<<<B, 64, 0, s>>>(out_dev, E);
    }
    const hipError_t e = hipEventRecord(h->done, s);
    if (rc) return rc;
    THIP(e);
    THIP(hipGetLastError());
    return 0;
}

int clipvit_text_destroy(clipvit_text_handle* h) {
    g_err.clear();
    if (!h) return 0;
    hipSetDevice(h->device);
    hipDeviceSynchronize();
    for (auto& kv : h->master) hipFree(kv.second);
    for (auto& l : h->layers) {
        hipFree(l.wqkv);
        hipFree(l.wout);
        hipFree(l.wfc);
        hipFree(l.wproj);
    }
    hipFree(h->scratch);
    hipFree(h->x);
    hipFree(h->h);
    hipFree(h->qkv);
    hipFree(h->u);
    hipFree(h->eot);
    if (h->done) hipEventDestroy(h->done);
    delete h;
    return 0;
}

}  // extern "C"
