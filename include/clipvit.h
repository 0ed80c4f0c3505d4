/*
 * clipvit.h — C ABI of libclipvit_hip.so, the MI355X (gfx950) CLIP-ViT image path.
 *
 * This library replaces, for the hot path only, the `(model, preprocess)` pair that the
 * reference obtains from `clip.load("ViT-B/16", device)` (main.py:152, main.py:241,
 * python-worker/main_API.py:137) and the cosine head that main.py computes around it.
 * Each entry point names the reference interface it stands in for.
 *
 * Conventions
 *   - every function returns int status: 0 = OK, negative = error; the message of the
 *     last error on the calling host thread is returned by clipvit_last_error().
 *   - "dev" pointers are device (HBM) pointers on the handle's device, owned by the caller.
 *   - a handle is pinned to one device; weights are immutable after loading, so
 *     encode/classify may be called concurrently from several host threads (each call
 *     takes a workspace from a mutex-guarded pool, ordered by HIP events).
 *   - stream arguments are hipStream_t passed as void*; NULL = the legacy default stream.
 *   - no torch types cross this boundary: plain pointers, sizes and enums only.
 */
#ifndef CLIPVIT_H
#define CLIPVIT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: clipvit_attention_test takes `causal` (8 arguments; version 1 had 7), and
 *    clipvit_profile_forward writes 20 floats to out_ms (version 1 wrote 10: a version-1 caller's
 *    10-float buffer overflows).
 * 3: clipvit_set_tuning (the library reads no environment variables).
 * 4: clipvit_gemm_log (test hook). */
#define CLIPVIT_ABI_VERSION 4

/* Status codes. */
#define CLIPVIT_OK 0
#define CLIPVIT_E_INVALID (-1)   /* bad argument / shape / name                         */
#define CLIPVIT_E_HIP (-2)       /* a HIP runtime call failed                           */
#define CLIPVIT_E_STATE (-3)     /* call out of order (e.g. classify before text feats) */
#define CLIPVIT_E_NOMEM (-4)     /* device allocation failed                             */

/* Element types of buffers crossing the ABI. */
typedef enum {
    CLIPVIT_F32 = 0,
    CLIPVIT_BF16 = 1,
    CLIPVIT_F16 = 2,
    CLIPVIT_MXFP8 = 3, /* compute_dtype only: MX-fp8 Linears (e4m3 + E8M0 per 32), bf16 elsewhere */
} clipvit_dtype;

/* Model geometry. Mirrors OpenAI-CLIP VisionTransformer(input_resolution, patch_size,
 * width, layers, heads, output_dim) as built by clip.load [3p] for the name passed at
 * main.py:152 / main.py:241.  compute_dtype selects the MFMA operand type (BF16 or F16, or
 * MXFP8: the 4 Linears of every block in MX-fp8 with bf16 attention / patch embedding);
 * the residual stream, LayerNorm statistics, softmax and the head stay fp32. */
typedef struct {
    int image_size;     /* 224 (B/32, B/16) or 336 (L/14@336)          */
    int patch_size;     /* 32, 16, 14                                   */
    int width;          /* 768 / 1024  (multiple of 256)                */
    int layers;         /* 12 / 24                                      */
    int heads;          /* width / 64                                   */
    int embed_dim;      /* 512 / 768   (multiple of 64)                 */
    int compute_dtype;  /* CLIPVIT_BF16, CLIPVIT_F16 or CLIPVIT_MXFP8    */
    int max_batch;      /* largest B accepted by encode/classify        */
} clipvit_config;

/* A host fp32 tensor keyed by its OpenAI-CLIP state-dict name (e.g.
 * "visual.transformer.resblocks.3.mlp.c_fc.weight"). Row-major, contiguous. */
typedef struct {
    const char* name;
    const float* data;
    int ndim;
    int64_t shape[4];
} clipvit_tensor;

/* One LoRA adapter to merge into a Linear of the vision tower.
 * Reference layout (main.py:19-31): lora_A [in, rank], lora_B [rank, out],
 * forward = linear(x) + (x @ A @ B) * scaling  with scaling = alpha / rank.
 * target = OpenAI name of the Linear's weight, e.g.
 * "visual.transformer.resblocks.0.attn.in_proj_weight" or "...mlp.c_fc.weight". */
typedef struct {
    const char* target;
    const float* A;   /* [in, rank]  host fp32 */
    const float* B;   /* [rank, out] host fp32 */
    int in_features;
    int out_features;
    int rank;
    float scaling;    /* alpha / rank */
} clipvit_lora;

typedef struct clipvit_handle clipvit_handle;

/* Replaces clip.load(name, device) model construction (main.py:152, main.py:241).
 * Allocates the weight store and the first workspace for cfg->max_batch images. */
int clipvit_create(const clipvit_config* cfg, int device, clipvit_handle** out);

/* Test / A-B hook, not part of the reference's surface: select one of the measured
 * alternatives DESIGN.md records instead of the shipped default, before clipvit_load_weights
 * (CLIPVIT_E_STATE after it). spec = "key=value;key=value", keys: resid16, defer_x, lnfold,
 * cls_prune, round_split, attn_q8, x16, x24, u_blocked (0/1); w_blocked (0/1/2: the Linear
 * weights also kept in the 16-row blocked layout, read by every tile that can (2, default) or
 * by the variant-72 / 74 launches only (1); 0 = no copies);
 * split_variants "main,tail"; tail_variant; tail_kmin (>= 64, multiple of 64) / tail_smax (1..48):
 * the class-token tail's split-K rule; head_cols (64 / 32); mx8_split_tail (0, 2, 5);
 * split_xcd; max_inflight; split_min (<= 0: never split); gemm_xcd / gemm_variants "q,o,f,p,e";
 * qkv_variant / fc_variant / out_variant / proj_variant (100 * XCD map + tile of that role only;
 * 79 = the 192 x 256 persistent tile for out_proj / c_proj); fc_balanced (0/1:
 * c_fc with >= 2 whole rounds of 256x256 tiles plus a remainder as one balanced launch, default 1,
 * or as the round split of split_variants); fc_balanced_variant (75 / 77: its tile);
 * h_blocked (0..3: ln_2 writes c_fc's A in the 16-row blocked layout by direct stores (1) or an
 * LDS transpose of 16-row (2) or 8-row (3, default) groups per workgroup); patch_im2col (0/1: the pixel cast writes a blocked im2col matrix
 * for an explicit patch GEMM, default 1; 0 = the implicit GEMM over the cast pixels);
 * ln1_rows (1/2: rows per wave of the add + LayerNorm after c_proj, default 1); attn_persist (0..4: N <= 64 attention as a persistent loop on that many workgroups per CU);
 * attn_fuse (0/1: ViT-B/32 blocks 0 .. L-2 as one attention + out_proj + add + ln_2 kernel per
 * image, default 0);
 * trace_gemm (0/1: clipvit_gemm_log);
 * large_variants "q,f,o,p"; mx8_variants "q,o,f,p" (3 = ping-pong 256x256, 4 = the 32x32x64 scaled-MFMA
 * form of the 32-deep-k-step tile, QKV / c_fc only); mx8_skip / mx8_skip_mlp "i,j,.." (bf16
 * blocks; mx8_skip sets both masks). An unknown key or bad value fails with CLIPVIT_E_INVALID
 * and leaves the handle unchanged. The product path never calls it. */
int clipvit_set_tuning(clipvit_handle* h, const char* spec);

/* Test hook (ABI 4), not part of the reference's surface: with tuning trace_gemm=1, every GEMM
 * launch of the encoder's Linear roles is logged as 4 ints {role (0 qkv, 1 out_proj, 2 c_fc,
 * 3 c_proj), tile variant, M, flags (1 blocked W copy, 2 MX-fp8, 4 blocked A, 8 blocked C)}.
 * Copies up to `cap` entries (4 * cap ints) to out, clears the log and returns the count. */
int clipvit_gemm_log(clipvit_handle* h, int* out, int cap);

/* Replaces the weight half of clip.load [3p]: host fp32 tensors keyed by OpenAI names.
 * The library copies them to HBM, keeps fp32 masters, and packs the MFMA operands.
 * Every visual.* tensor of the geometry must be present (text-tower names are ignored). */
int clipvit_load_weights(clipvit_handle* h, const clipvit_tensor* tensors, size_t n);

/* Replaces replace_linears_with_lora + load_lora_weights_to_model (main.py:62-113) for the
 * vision tower: W' = W + scaling * (A @ B)^T merged into the fp32 master, then re-packed.
 * Linears with no adapter keep a zero delta (lora_B = 0 init, main.py:27). Runtime cost 0. */
int clipvit_load_lora(clipvit_handle* h, const clipvit_lora* items, size_t n);

/* Replaces the cached text matrices of InteriorImageDetector (main.py:179-182) and
 * CachedInteriorAnalyzer._precompute_text_features_optimized (main.py:296-311):
 * T [C, E] host fp32 rows (already L2-normalised by the caller, as the reference does),
 * split into nseg consecutive segments by seg_offsets[0..nseg] (seg_offsets[0] = 0,
 * seg_offsets[nseg] = C). Softmax and top-k run independently per segment. */
int clipvit_set_text_features(clipvit_handle* h, const float* T, int C, int E,
                              const int* seg_offsets, int nseg);

/* Replaces model.encode_image(x) (main.py:204, main.py:444, main.py:503).
 * pixels_dev: [B, 3, R, R] CLIP-normalised pixels of `dtype`; emb_dev: [B, E] fp32,
 * the projected image features BEFORE L2 normalisation (what encode_image returns). */
int clipvit_encode_image(clipvit_handle* h, void* stream, const void* pixels_dev, int dtype,
                         int B, float* emb_dev);

/* Replaces encode_image + the head of main.py:205-217 / 445-459 / 504-509:
 *   f = encode_image(x); f /= ||f||; logits = 100 * f @ T^T; per segment softmax + topk(min(5,n)).
 * Outputs (any may be NULL except logits):
 *   emb_dev    [B, E]      fp32, L2-normalised features
 *   logits_dev [B, C]      fp32
 *   probs_dev  [B, C]      fp32, softmax within each segment
 *   top_idx    [B, nseg, 5] int32 column index inside the segment (-1 where n < 5)
 *   top_prob   [B, nseg, 5] fp32 */
int clipvit_classify(clipvit_handle* h, void* stream, const void* pixels_dev, int dtype, int B,
                     float* emb_dev, float* logits_dev, float* probs_dev, int32_t* top_idx,
                     float* top_prob);

/* Number of text classes / segments currently set (0 if none). */
int clipvit_text_shape(clipvit_handle* h, int* C, int* nseg);

/* Frees every device allocation of the handle. */
int clipvit_destroy(clipvit_handle* h);

/* Thread-local message of the last failing call on this host thread ("" if none). */
const char* clipvit_last_error(void);

/* ABI version compiled into the library (CLIPVIT_ABI_VERSION). */
int clipvit_abi_version(void);

/* ---- Text tower ----
 * Replaces model.encode_text(clip.tokenize(prompts)) [3p] as run once per prompt set by
 * InteriorImageDetector (main.py:179-182) and CachedInteriorAnalyzer.
 * _precompute_text_features_optimized (main.py:296-311); its normalised output is the T that
 * clipvit_set_text_features takes. Geometry mirrors CLIP(transformer_width, _layers, _heads,
 * context_length, vocab_size, embed_dim) [3p]. */
typedef struct {
    int width;          /* 512 (B models) / 768 (L/14), multiple of 256 */
    int layers;         /* 12                                          */
    int heads;          /* width / 64                                  */
    int context;        /* 77                                          */
    int vocab;          /* 49408 for the OpenAI BPE vocabulary          */
    int embed_dim;      /* 512 / 768 (multiple of 64)                   */
    int compute_dtype;  /* CLIPVIT_BF16 or CLIPVIT_F16                  */
    int max_batch;      /* prompts per encode call                     */
} clipvit_text_config;

typedef struct clipvit_text_handle clipvit_text_handle;

/* Text-tower model construction (the text half of clip.load, main.py:152 / main.py:241). */
int clipvit_text_create(const clipvit_text_config* cfg, int device, clipvit_text_handle** out);

/* Host fp32 tensors keyed by OpenAI names: token_embedding.weight [vocab, W],
 * positional_embedding [context, W], transformer.resblocks.{i}.* (same leaves as the vision
 * blocks), ln_final.{weight,bias}, text_projection [W, E]. visual.* names are ignored. */
int clipvit_text_load_weights(clipvit_text_handle* h, const clipvit_tensor* tensors, size_t n);

/* Replaces the text half of replace_linears_with_lora + load_lora_weights_to_model
 * (main.py:62-113, main.py:247-251): targets "transformer.resblocks.{i}.mlp.c_fc.weight" etc.
 * (where the shipped comprehensive_lora*.pth adapters bind). Same merge rule and reset
 * semantics as clipvit_load_lora. */
int clipvit_text_load_lora(clipvit_text_handle* h, const clipvit_lora* items, size_t n);

/* Replaces model.encode_text(tokens) (main.py:181, main.py:308), optionally followed by the
 * L2 normalisation of main.py:182 / main.py:309. tokens_dev: [B, context] int32 ids as
 * clip.tokenize produces (sot ... eot, zero padded; pooled at the argmax id = eot);
 * out_dev: [B, embed_dim] fp32. Ids outside [0, vocab) are clamped. */
int clipvit_encode_text(clipvit_text_handle* h, void* stream, const int32_t* tokens_dev, int B,
                        int l2_normalize, float* out_dev);

int clipvit_text_destroy(clipvit_text_handle* h);

/* ---- GPU preprocessing ----
 * Replaces preprocess(img) = clip's _transform(n_px) [3p] at main.py:201, main.py:438,
 * main.py:489 for images already decoded to RGB (load_image, main.py:119-128):
 * Resize(n_px, BICUBIC) -> CenterCrop(n_px) -> ToTensor -> Normalize(CLIP mean/std).
 * The resampling is Pillow's 8-bit fixed-point two-pass convolution, bit-identical to
 * PIL.Image.resize(BICUBIC) followed by the crop. */
typedef struct {
    int64_t offset;   /* byte offset of the image's HWC uint8 RGB pixels in rgb_dev */
    int width;        /* source width  (pixels) */
    int height;       /* source height (pixels) */
} clipvit_image;

/* B images packed in one device byte buffer (each image [height, width, 3] uint8 at its
 * offset) -> out_dev [B, 3, n_px, n_px] CLIP-normalised pixels of out_dtype (F32, BF16 or
 * F16), the input clipvit_encode_image / clipvit_classify take. Asynchronous on `stream`;
 * the image table is staged before the call returns, so `images` may be freed after it. */
int clipvit_preprocess(void* stream, const unsigned char* rgb_dev, const clipvit_image* images,
                       int B, int n_px, int out_dtype, void* out_dev);

/* Host-only: Pillow's resampling plan for one axis (in_size -> out_size, bicubic): *ksize
 * taps per output; bounds [out_size][2] = (first source index, tap count); kk
 * [out_size][*ksize] fixed-point weights with 22 fraction bits (kk_cap = capacity of kk in
 * int32 elements). Identity plan (1 tap, weight 2^22) when in_size == out_size. */
int clipvit_resample_plan(int in_size, int out_size, int* ksize, int* bounds, int32_t* kk,
                          int kk_cap);

/* ---- kernel-level entry points (testing / benchmarking of single hot kernels) ----
 * These operate on caller-owned device buffers with the packed layouts documented in
 * DESIGN.md; they are what the per-kernel parity tests and the roofline probe call. */

/* C[M,N] = A[M,K] @ W[N,K]^T + bias.  A_dev: 16-bit (`dtype` BF16/F16) row-major;
 * W_dev: fp32 [N,K] natural row order (packed to `dtype` internally, as clipvit_load_weights
 * does); bias fp32 [N] or NULL; C fp32 [M,N]. epi: 0 = store, 1 = QuickGELU then store,
 * 2 = accumulate into C (residual add), 10 / 11 = 16-bit store / QuickGELU widened to fp32,
 * 20 + S = split-K into S slices (pipelined variants >= 8; C holds [S][M][N] fp32 partial
 * products without bias; K % (64 S) == 0 — the class-token tail's GEMMs). K % 64 == 0, N % 64 == 0 (N % 128 for variants 1-2,
 * N % 256 for variant 3). variant % 100 selects the tile kernel (0 auto; the table in
 * csrc/gemm.hip pick/launch_gemm); variant / 100 the block->XCD mapping
 * (0/1 = 1-D bijective remap, 2 = 4x2 (M-band, N-half) partition; pipelined variants only);
 * + 10000 = W in the 16-row blocked layout, + 20000 = A blocked, + 30000 = both.
 * The same encoding applies to clipvit_gemm_bench. */
int clipvit_gemm_test(void* stream, int dtype, const void* A_dev, const void* W_dev,
                      const float* bias_dev, float* C_dev, int M, int N, int K, int epi,
                      int variant);

/* Average device time (ms) of `iters` back-to-back launches of one GEMM on random uniform
 * [-1,1) operands allocated inside (tile-variant tuning; epi = internal epilogue enum:
 * 0 store16, 1 gelu16, 2 resid32, 3 patch32, 4 f32, 5 f32gelu). Default stream. */
int clipvit_gemm_bench(int dtype, int M, int N, int K, int epi, int variant, int iters,
                       float* avg_ms);

/* MX-fp8 quantization of a row-major [rows, K] buffer (in_dtype F32/BF16/F16, K % 32 == 0):
 * q [rows, K] OCP e4m3 bytes, sq [rows, K/32] E8M0 block scales (block = 32 consecutive
 * columns; scale exponent = smallest e with amax * 2^-e <= 448, clamped to [-127, 126]). */
int clipvit_quant_mx8_test(void* stream, int in_dtype, const void* src_dev, int rows, int K,
                           unsigned char* q_dev, unsigned char* sq_dev);

/* MX-fp8 GEMM: A = (A8 [M,K] e4m3, sA [M,K/32]); W fp32 [N,K] natural order (quantized and
 * packed internally by the load-time packer); bias fp32 [N] or NULL. K % 128 == 0,
 * N % 128 == 0. epi: 0 C fp32 = A W^T + b; 1 QuickGELU of that; 2 C fp32 += A W^T + b;
 * 3 C = MX-fp8 of (A W^T + b) [M,N] bytes with scales sC [M,N/32]; 4 = 3 after QuickGELU;
 * 5 C bf16 [M,N]. variant: 0 auto, 1 128x256, 2 128x128; + 100 * XCD partition. */
int clipvit_gemm_mx8_test(void* stream, const unsigned char* A8_dev, const unsigned char* sA_dev,
                          const float* W_dev, const float* bias_dev, void* C_dev,
                          unsigned char* sC_dev, int M, int N, int K, int epi, int variant);

/* The 24-bit residual stream format of the 16-bit forward: x fp32 [n] (n % 4 == 0)
 * -> planes [3n bytes: n u16 upper halves, then n bytes of the next 8 mantissa bits, rounded to
 * nearest at bit 8] -> back fp32 [n], by the kernels' own encode / decode functions. */
int clipvit_residual_x24_test(void* stream, const float* x_dev, void* planes_dev, float* back_dev, size_t n);

/* softmax(Q K^T / sqrt(64)) V for a packed qkv [B*N, 3*H*64] buffer of `dtype`;
 * out [B*N, H*64] of `dtype`. causal bit 0: key j masked for query i < j (the text tower);
 * causal >> 4 = k > 0 with N <= 64: the persistent one-key-block kernel on k workgroups per CU
 * (tuning attn_persist). */
int clipvit_attention_test(void* stream, int dtype, const void* qkv_dev, void* out_dev, int B,
                           int N, int H, int causal);

/* Time `iters` launches of ONE lane's encoder forward (the per-stream batch the call path
 * launches for B images: ceil(B/2) when the batch is split over the two lane streams, else B)
 * serialised on `stream`, with a HIP event closing every kernel-family interval; out_ms must
 * hold 20 floats:
 *   out_ms[0..8]   average device time (ms) per family and forward: 0 patch+embed, 1 qkv gemm,
 *                  2 attention, 3 out-proj gemm, 4 layernorm, 5 fc gemm, 6 proj gemm, 7 head
 *                  (ln_post+proj), 8 the last block's row-wise part on class-token rows (0 when
 *                  the full last block runs);
 *   out_ms[9]      the lane batch profiled;
 *   out_ms[10..18] event intervals per family and forward (same order as 0..8);
 *   out_ms[19]     device time (ms) between two back-to-back events with no work between them
 *                  (the per-interval cost of the marks, included in out_ms[0..8]).
 * Requires weights loaded. Used by bench.py's roofline probe. (ABI version 2.) */
int clipvit_profile_forward(clipvit_handle* h, void* stream, const void* pixels_dev, int dtype,
                            int B, int iters, float* out_ms);

#ifdef __cplusplus
}
#endif
#endif /* CLIPVIT_H */
