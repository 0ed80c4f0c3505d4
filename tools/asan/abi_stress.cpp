// Host-side sanitizer run of libclipvit_hip.so's C ABI (SURVEY.md §5 "race detection /
// sanitizers": the reference's 4 detector threads on one shared model, main.py:345-346).
// Built by tools/asan/build.sh with -Xarch_host -fsanitize=address,undefined on every host
// translation unit of the library and on this driver (device code is not instrumented).
// Runs ViT-B/32 with synthetic weights: create -> load_weights -> load_lora -> set_text_features
// -> 4 threads x 6 classify calls (each thread its own stream and buffers) -> bad-argument
// calls (each must return an error, not crash) -> destroy. Exit 0 = no sanitizer report and
// every thread's logits equal thread 0's.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "clipvit.h"

#define CK(x)                                                                                 \
    do {                                                                                      \
        int rc_ = (x);                                                                        \
        if (rc_) {                                                                            \
            std::fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,       \
                         clipvit_last_error());                                               \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

struct Host {
    std::string name;
    std::vector<float> v;
    std::vector<int64_t> shape;
};

int main() {
    const int D = 768, L = 12, E = 512, P = 32, R = 224, N = 50, B = 8, C = 437;
    clipvit_config cfg{R, P, D, L, D / 64, E, CLIPVIT_F16, B};
    clipvit_handle* h = nullptr;
    CK(clipvit_create(&cfg, 0, &h));

    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<Host> ts;
    auto add = [&](const std::string& n, std::vector<int64_t> s, float scale, float offset = 0.f) {
        size_t cnt = 1;
        for (auto d : s) cnt *= (size_t)d;
        Host t{n, std::vector<float>(cnt), s};
        for (auto& x : t.v) x = offset + scale * nd(rng);
        ts.push_back(std::move(t));
    };
    add("visual.conv1.weight", {D, 3, P, P}, 0.02f);
    add("visual.class_embedding", {D}, 0.036f);
    add("visual.positional_embedding", {N, D}, 0.036f);
    add("visual.ln_pre.weight", {D}, 0.f, 1.f);
    add("visual.ln_pre.bias", {D}, 0.f);
    for (int i = 0; i < L; ++i) {
        const std::string p = "visual.transformer.resblocks." + std::to_string(i) + ".";
        add(p + "ln_1.weight", {D}, 0.f, 1.f);
        add(p + "ln_1.bias", {D}, 0.f);
        add(p + "attn.in_proj_weight", {3 * D, D}, 0.02f);
        add(p + "attn.in_proj_bias", {3 * D}, 0.f);
        add(p + "attn.out_proj.weight", {D, D}, 0.02f);
        add(p + "attn.out_proj.bias", {D}, 0.f);
        add(p + "ln_2.weight", {D}, 0.f, 1.f);
        add(p + "ln_2.bias", {D}, 0.f);
        add(p + "mlp.c_fc.weight", {4 * D, D}, 0.02f);
        add(p + "mlp.c_fc.bias", {4 * D}, 0.f);
        add(p + "mlp.c_proj.weight", {D, 4 * D}, 0.02f);
        add(p + "mlp.c_proj.bias", {D}, 0.f);
    }
    add("visual.ln_post.weight", {D}, 0.f, 1.f);
    add("visual.ln_post.bias", {D}, 0.f);
    add("visual.proj", {D, E}, 0.036f);
    std::vector<clipvit_tensor> tv;
    for (auto& t : ts) {
        clipvit_tensor x{};
        x.name = t.name.c_str();
        x.data = t.v.data();
        x.ndim = (int)t.shape.size();
        for (int k = 0; k < x.ndim; ++k) x.shape[k] = t.shape[k];
        tv.push_back(x);
    }
    CK(clipvit_load_weights(h, tv.data(), tv.size()));

    // LoRA r=8 on c_fc of block 0 (A [in, r], B [r, out])
    const int r = 8;
    std::vector<float> A((size_t)D * r), Bm((size_t)r * 4 * D);
    for (auto& x : A) x = 0.02f * nd(rng);
    for (auto& x : Bm) x = 0.01f * nd(rng);
    clipvit_lora lo{"visual.transformer.resblocks.0.mlp.c_fc.weight", A.data(), Bm.data(), D, 4 * D, r, 2.f};
    CK(clipvit_load_lora(h, &lo, 1));

    std::vector<float> T((size_t)C * E);
    for (int c = 0; c < C; ++c) {
        double n2 = 0;
        for (int e = 0; e < E; ++e) n2 += (T[(size_t)c * E + e] = nd(rng)) * (double)T[(size_t)c * E + e];
        for (int e = 0; e < E; ++e) T[(size_t)c * E + e] /= (float)std::sqrt(n2);
    }
    const int seg[7] = {0, 40, 60, 359, 395, 425, 437};
    CK(clipvit_set_text_features(h, T.data(), C, E, seg, 6));

    std::vector<float> px((size_t)B * 3 * R * R);
    for (auto& x : px) x = std::fmin(2.2f, std::fmax(-1.8f, nd(rng)));
    void* dpx = nullptr;
    if (hipMalloc(&dpx, px.size() * 4) != hipSuccess) return 1;
    if (hipMemcpy(dpx, px.data(), px.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return 1;

    const int NT = 4, IT = 6;
    std::vector<std::vector<float>> got(NT, std::vector<float>((size_t)B * C));
    std::vector<int> status(NT, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < NT; ++t)
        th.emplace_back([&, t] {
            hipStream_t s;
            float *lg = nullptr, *pr = nullptr, *tp = nullptr, *em = nullptr;
            int32_t* ti = nullptr;
            if (hipStreamCreate(&s) != hipSuccess || hipMalloc(&lg, (size_t)B * C * 4) != hipSuccess ||
                hipMalloc(&pr, (size_t)B * C * 4) != hipSuccess || hipMalloc(&em, (size_t)B * E * 4) != hipSuccess ||
                hipMalloc(&ti, (size_t)B * 6 * 5 * 4) != hipSuccess || hipMalloc(&tp, (size_t)B * 6 * 5 * 4) != hipSuccess) {
                status[t] = 1;
                return;
            }
            for (int i = 0; i < IT && !status[t]; ++i)
                status[t] = clipvit_classify(h, s, dpx, CLIPVIT_F32, B, em, lg, pr, ti, tp);
            if (!status[t] && hipStreamSynchronize(s) == hipSuccess)
                status[t] = hipMemcpy(got[t].data(), lg, (size_t)B * C * 4, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
            hipFree(lg); hipFree(pr); hipFree(em); hipFree(ti); hipFree(tp);
            hipStreamDestroy(s);
        });
    for (auto& x : th) x.join();
    for (int t = 0; t < NT; ++t) {
        if (status[t]) {
            std::fprintf(stderr, "thread %d: status %d (%s)\n", t, status[t], clipvit_last_error());
            return 1;
        }
        if (std::memcmp(got[t].data(), got[0].data(), got[0].size() * 4) != 0) {
            std::fprintf(stderr, "thread %d: logits differ from thread 0\n", t);
            return 1;
        }
    }
    // error paths: each must fail with a status, not crash
    int bad = 0;
    bad += clipvit_classify(h, nullptr, dpx, CLIPVIT_F32, B + 1, nullptr, (float*)dpx, nullptr, nullptr, nullptr) != 0;
    bad += clipvit_classify(h, nullptr, nullptr, CLIPVIT_F32, B, nullptr, (float*)dpx, nullptr, nullptr, nullptr) != 0;
    bad += clipvit_classify(h, nullptr, dpx, 7, B, nullptr, (float*)dpx, nullptr, nullptr, nullptr) != 0;
    clipvit_tensor wrong = tv[0];
    wrong.shape[0] = D + 1;
    bad += clipvit_load_weights(h, &wrong, 1) != 0;
    clipvit_lora badl = lo;
    badl.target = "visual.transformer.resblocks.99.mlp.c_fc.weight";
    bad += clipvit_load_lora(h, &badl, 1) != 0;
    if (bad != 5) {
        std::fprintf(stderr, "error paths: %d of 5 rejected\n", bad);
        return 1;
    }
    CK(clipvit_destroy(h));
    hipFree(dpx);
    std::printf("abi_stress ok: %d threads x %d classify calls, identical logits; 5 bad calls rejected\n", NT, IT);
    std::fflush(stdout);  // LeakSanitizer's exit path does not flush stdio
    return 0;
}
