// libclipvit_hip.so — host side of the C ABI declared in include/clipvit.h.
//
// Owns the device weight store (fp32 masters + packed 16-bit MFMA operands), merges LoRA at
// load time, keeps the text-feature table, and runs the encoder forward as a fixed sequence of
// hand-written gfx950 kernels on the caller's stream:
//
//   implicit-GEMM patch embedding (pixels -> LDS patch tiles, EPI_PATCH) -> embed+ln_pre+ln_1
//   12x [ GEMM(qkv) -> attention -> GEMM(out_proj, +residual) -> ln_2
//         -> GEMM(c_fc, QuickGELU) -> GEMM(c_proj, +residual) -> ln_1(next) ]
//   -> ln_post(CLS) @ proj -> [classify: L2-norm, 100*cos logits, segment softmax, top-5]
//
// Reference call sites replaced: clip.load (main.py:152, 241), encode_image (main.py:204,
// 444, 503), LoRA injection + loading (main.py:62-113, 247-251), text caches (main.py:179-182,
// 296-311) and the head (main.py:205-217, 445-459, 504-509).
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "clipvit.h"
#include "common.h"

namespace clipvit {
// last error of this host thread; shared with preprocess.hip
thread_local std::string g_err;
}  // namespace clipvit

using namespace clipvit;

#define FAIL(code, msg)        \
    do {                       \
        g_err = (msg);         \
        return (code);         \
    } while (0)

#define HIPCHK(x)                                                                  \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            g_err = std::string(#x) + " failed: " + hipGetErrorString(e_);        \
            return CLIPVIT_E_HIP;                                                  \
        }                                                                          \
    } while (0)

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) hipSetDevice(prev);
    }
};

struct LayerW {
    void *wqkv = nullptr, *wout = nullptr, *wfc = nullptr, *wproj = nullptr;
    // the Linear weights again in the 16-row blocked layout (GemmArgs.blk_w), with w_blocked
    void *wqkv_b = nullptr, *wfc_b = nullptr, *wout_b = nullptr, *wproj_b = nullptr;
    const float *bqkv, *bout, *bfc, *bproj, *ln1g, *ln1b, *ln2g, *ln2b;
    // LayerNorm fold (lnfold): ln_1 into QKV, ln_2 into c_fc: s_n = sum_k W'_nk, b' = b + W beta
    float *s_qkv = nullptr, *bf_qkv = nullptr, *s_fc = nullptr, *bf_fc = nullptr;
};

// One lane = the activation buffers for `cap` images + the HIP stream that runs them.
struct Lane {
    int cap = 0;
    float* x = nullptr;  // [cap*N, D] fp32 residual stream
    void* h = nullptr;   // [cap*N, D] 16-bit LN output; also the attention output
    void* qkv = nullptr; // [cap*N, 3D]
    void* u = nullptr;   // [cap*N, 4D] MLP hidden; also the 16-bit pixel copy of a cast input
    float* f = nullptr;  // [cap, E] projected features
    float2* st = nullptr;  // lnfold: [cap*N, D/128] per-row 128-column (mean, M2) of x
    unsigned char* q8 = nullptr;  // MX-fp8 mode: [cap*N, D] e4m3 GEMM operand + [cap*N, D/32] scales
    void* x16 = nullptr;  // MX-fp8 mode: [cap*N, D] fp16 residual stream (handle x16)
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;  // recorded after the last kernel that touched the buffers
};

// A workspace slot serves one call at a time. A batch of B >= SPLIT_MIN images runs as two
// independent halves on the two lane streams (forked from / joined into the caller's stream
// by events), so one half's memory-bound kernels and GEMM tails overlap the other half's
// GEMMs. Smaller batches run on the caller's stream with lane 0.
constexpr int kLanes = 2;
// Default: split batches of at least SPLIT_IMAGES images and SPLIT_TOKENS tokens (B/32: 512
// images; B/16 and L/14@336: 130 / 128). B/32 at bs 256 stays on one stream: there the split
// won on some boxes and lost on others, and its half-batch launches make the per-kernel
// roofline ill-defined. Measured on MI355X (round 2, alternating A/B, same box):
// B/32 bs 256 fp16 78.7k -> 80.8k and 78.2k -> 81.0k img/s on two boxes, 82.6k -> 82.1k on a
// faster one; bf16 bs 512 81.5k -> 86.8k and 84.1k -> 87.0k; MX-fp8 bs 512 93.0k -> 99.0k;
// L/14@336 bs 128 2,183 -> 2,269 and 2,179 -> 2,280; B/16 bs 256 21.25k -> 21.43k. Smaller
// batches lose (B/32 bs 64 39.4k -> 38.2k, B/16 bs 64 20.3k -> 19.6k). Round 1 measured a loss
// at bs 256 with the earlier tile table. tuning split_min=n overrides (<= 0: never split).
constexpr int SPLIT_NEVER = 1 << 30;
constexpr int SPLIT_TOKENS = 25600, SPLIT_IMAGES = 128;
struct Workspace {
    Lane lane[kLanes];
    hipEvent_t fork = nullptr;
    bool used = false;
    hipStream_t last_stream = nullptr;  // stream of the last call that used it
    unsigned long long last_use = 0;    // call counter at that use (LRU)
};

// F_TAIL: the last block's row-wise part on class-token rows (cls_tail)
enum Fam { F_EMBED = 0, F_QKV, F_ATTN, F_OUT, F_LN, F_FC, F_PROJ, F_HEAD, F_TAIL, F_COUNT };

struct Prof {
    std::vector<hipEvent_t> ev;
    std::vector<int> fam;
    size_t k = 0;
    void mark(hipStream_t s, int f) {
        if (k < ev.size()) {
            hipEventRecord(ev[k], s);
            fam[k] = f;
            ++k;
        }
    }
};

}  // namespace

struct clipvit_handle {
    clipvit_config cfg{};
    int device = 0;
    int G = 0, G2 = 0, N = 0, D = 0, E = 0, K3 = 0, Kp = 0, dt = 1;
    std::unordered_map<std::string, float*> master;
    std::unordered_map<std::string, std::vector<int64_t>> shapes;
    std::vector<std::string> order;
    void* wpatch = nullptr;
    void* wpatch_b = nullptr;  // its 16-row blocked copy (the explicit patch GEMM, patch_im2col)
    std::vector<LayerW> layers;
    float* scratch = nullptr;
    size_t scratch_elems = 0;
    bool loaded = false;
    // cached pointers into `master` (read concurrently by forward(); never via operator[])
    const float *cls = nullptr, *pos = nullptr, *lnpre_g = nullptr, *lnpre_b = nullptr;
    const float *lnpost_g = nullptr, *lnpost_b = nullptr, *proj = nullptr;
    float* Tt = nullptr;
    int C = 0, Cpad = 0, nseg = 0;
    int* seg_dev = nullptr;
    std::vector<int> seg_host;
    std::mutex mu;
    std::vector<Workspace*> pool;
    // GEMM tile variants per role (qkv, out, fc, proj, patch), from in-model sweeps on MI355X
    // (profiles/ablog.md; tools/ab_envs.sh); tuning gemm_variants="q,o,f,p,e".
    // 22 = 160x128 tiles of 4 waves, two workgroups per CU (the N = 768 roles). The 224x192
    // one-round tiles 92 / 93 win standalone (c_proj 67.4 -> 62.7 us, patch 75.2 -> 69.6) but
    // not in-model (c_proj 0.777 -> 0.785-0.81 ms per forward, patch 0.134 -> 0.143-0.158).
    // 98 = 240x256 QKV tiles of 12 waves (486 tiles = 1.9 rounds at bs 256 against 450 = 1.76
    // of 256x256): in-model QKV 0.673 -> 0.662 ms per forward. c_fc on 22 in one launch since
    // the 4-wave tiles keep their accumulators in VGPRs (gemm_pipe_kernel launch bounds): c_fc
    // 0.795 ms per forward as with the round split (8 + 81), c_proj after it 0.675 -> 0.658 ms,
    // B/32 bs 256 85.6k -> 86.3k img/s (2 same-box alternations). r06: QKV on the 32-deep-k-step
    // tile (72) with its A in the blocked layout (qkv_blk): QKV family 0.626 -> 0.615 ms per
    // forward on 72 alone, 0.580 -> 0.560 with the blocked A (profiles/r06/qkv_ab.txt)
    int var[5] = {72, 82, 22, 82, 22};
    bool var_forced = false;  // tuning gemm_variants given: no shape-based override
    // tile of the QKV / c_fc roles at large M (>= 4 rounds of 256x256 tiles), 100 * XCD map +
    // tile; 0 = the 2-phase 256x256 tile (8). Default: the persistent ping-pong tile with the
    // column-group-major map (3462, gemm_pp.hip): B/16 22.3k -> 23.0k img/s, L/14@336 2,322 ->
    // 2,388 (same-box A/B, profiles/design_r05.md §5.8); c_fc with non-temporal output stores (3463): its
    // family 7.49 -> 7.03 ms per L/14 lane forward; out_proj / c_proj on 3463 too: L/14@336
    // 2,392-2,396 -> 2,416 img/s (B/16 unchanged). r05: the 32-deep-k-step tile (3472, gemm_p32.h)
    // on every role with QKV / c_fc reading their blocked weight copies (w_blk): L/14@336 bs 128
    // 2,406 / 2,407 -> 2,526 / 2,529 img/s (same box, profiles/r05/l14_ab.txt); c_fc with
    // non-temporal stores (3474: its u no longer sits dirty in front of the next QKV): L/14
    // 2,522 / 2,586 -> 2,614 / 2,613, B/16 24.1k / 24.2k -> 24.5k / 24.5k (profiles/r05/nt_*).
    // tuning large_variants="q,f,o,p"
    int large_var[4] = {3472, 3474, 3472, 3472};  // QKV, c_fc, out_proj, c_proj
    int ncu = 256;            // compute units of the device
    // tile->XCD partition per role (tuning gemm_xcd="q,o,f,p,e"): 2 = 4x2 (M, N) XCD grid,
    // 0/1 = 1-D bijective remap. out_proj / c_proj use the 1-D remap: same speed as the 4x2 grid
    // (c_proj 69.9 vs 70.0 us, out 24.0 vs 24.1) with each A panel read by one XCD instead of
    // two: PMC bytes / algorithmic 1.61 -> 1.13 (c_proj) and 1.33 -> 1.02 (out_proj)
    int xcd[5] = {0, 0, 2, 0, 1};
    int split_min = SPLIT_NEVER;  // batch size from which the two lane streams are used (clipvit_create)
    // MX-fp8 mode (compute_dtype CLIPVIT_MXFP8): the four Linears of every block run as
    // MX-fp8 GEMMs (packed weight = N*Kp e4m3 bytes followed by N*Kp/32 E8M0 scales);
    // patch embedding, attention and everything else stay bf16 / fp32.
    bool mx8 = false;
    // MX-fp8 GEMM tile per role (qkv, out, fc, proj); tuning mx8_variants. 128x128 everywhere:
    // measured at M = 25,600 (bs 512) qkv 88 -> 80 us, c_fc 110 -> 103 us against 128x256
    // out_proj on 160x128 (5): 480 tiles = one round at two per CU where 128x128 needs 1.17
    // (M = 12,800: 18.2 -> 15.1 us standalone, config 5 +1.7-2.3 % same box). c_fc on the
    // persistent ping-pong: 51.3 -> 55.8 us standalone, yet config 5 +1.5 % on two boxes (under
    // the two-lane split a kernel is priced by the CU time it holds)
    int var8[4] = {3, 5, 3, 3};  // QKV, out_proj, c_fc, c_proj: 3 = ping-pong 256x256 (mx8.hip)
    // MX c_fc whole-round row split (gemm8): tile of the tail launch (2 = 128x128, 5 = 160x128;
    // 0 = off: one launch); tuning mx8_split_tail. Off: the c_fc family is 6-8 % faster per
    // lane-forward with it (0.79 vs 0.85 ms), but config 5 runs two lanes and the tail's two
    // workgroups per CU hold CUs the other lane would use: 117.4k / 117.7k img/s with the split
    // against 117.9k / 118.6k without (same box, profiles/r04_ab3.txt)
    int mx8_split_tail = 0;
    // blocks kept in bf16 in MX-fp8 mode (bit i = block i); default the first two and last two
    // (measured: config-5 logit deviation 2.0e-2 with every block MX-fp8, 1.7e-2 with these
    // four in bf16 — DESIGN.md §5.6); tuning mx8_skip="..." overrides
    uint64_t mx8_skip = 0;
    // blocks whose MLP (c_fc, c_proj) stays bf16: the attention roles (QKV, out_proj) follow
    // mx8_skip, the MLP roles this mask (tuning mx8_skip sets both, mx8_skip_mlp this one):
    // the MLP GEMMs carry most of the MX-fp8 error, QKV / out_proj little of it
    uint64_t mx8_skip_mlp = 0;
    bool q8_attn(int i) const { return mx8 && !((mx8_skip >> i) & 1); }
    bool q8_mlp(int i) const { return mx8 && !((mx8_skip_mlp >> i) & 1); }
    // residual adds of out_proj / c_proj: true = the GEMM stores its 16-bit branch output y and
    // the following LayerNorm kernel does x += y (fp16 and bf16 default, set in clipvit_create; tuning resid16);
    // false = fp32 read-modify-write of x in the GEMM epilogue
    bool resid16 = false;
    // deferred residual store (fp16 path, see forward()); tuning defer_x=0 disables
    bool defer_x = true;
    // LayerNorm fold (tuning lnfold=1, fp16 only): ln_1 / ln_2
    // become per-row statistics written by the residual producers' epilogues (out_proj, c_proj,
    // embedding) and an affine correction in the QKV / c_fc epilogues; no LayerNorm pass
    bool lnfold = false;
    float* scratch2 = nullptr;  // W diag(gamma) staging for the folded Linears
    // last block on class-token rows only (see cls_tail); tuning cls_prune=0 disables
    bool cls_prune = true;
    unsigned long long calls = 0;  // acquire_ws counter (workspace LRU)
    int max_inflight = 2;  // workspaces kept for calls in flight on different streams (tuning max_inflight)
    int tail_var = 90;  // GEMM tile of the class-token tail (64x64, 4-stage ring; tuning tail_variant)
    // split-K of the class-token tail's GEMMs: the most slices (<= tail_smax, dividing K / 64)
    // that leave every slice >= tail_kmin deep (tuning tail_kmin / tail_smax)
    int tail_kmin = 192, tail_smax = 8;
    // output columns per workgroup of the head products (tuning head_cols 64 / 32, bit-identical):
    // 32 doubles the workgroups of ln_post @ proj (128 -> 256 at bs 256); head family 0.020 ->
    // 0.018-0.019 ms per forward, 3 alternations on one box (profiles/ablog.md)
    int head_cols = 32;
    // whole-round row split of c_fc (gemm()): the persistent ping-pong tile on the rows that fill
    // whole rounds, the 128x128 tile on the rest. r03, same box: B/32 82.0k / 82.1k -> 82.9k /
    // 83.0k img/s (c_fc 0.83 -> 0.80 ms per forward)
    // MX-fp8 forward, fp16 residual stream: the residual x lives in fp16 between the LayerNorm
    // kernels (which add and normalise in fp32) instead of fp32, halving their x bytes
    // (LayerNorm family = 30 % fewer HBM bytes). Needs the deferred 16-bit branch path and a
    // 16-bit class-token tail (the tail widens the class rows to fp32). tuning x16=0: fp32 x.
    bool x16 = true;
    // 16-bit forward (fp16 / bf16), 24-bit residual stream: x between the LayerNorm kernels as
    // 16 + 8 bit planes (norm.hip x24_load) instead of fp32: the add + LayerNorm kernels move 3
    // bytes per element of x instead of 4 (tuning x24=0: fp32 x). With lnfold the planes are read
    // and written by the residual producers' EPI_RES_STATS epilogues (GemmArgs.x24_plane)
    bool x24 = true;
    bool use_x24() const { return x24 && !mx8 && cls_prune && (lnfold || (resid16 && defer_x)); }
    bool use_x16() const {
        return x16 && mx8 && resid16 && defer_x && cls_prune && ((mx8_skip >> (cfg.layers - 1)) & 1) &&
               ((mx8_skip_mlp >> (cfg.layers - 1)) & 1);
    }
    // MX-fp8 forward: attention writes the out_proj operand (MX-fp8) itself instead of 16-bit
    // output + launch_quant_mx8 (same bytes; tuning attn_q8=0 restores the two kernels)
    bool attn_q8 = true;
    // ViT-B/32 on the 24-bit residual path: attention + out_proj + (x += y) + ln_2 of blocks
    // 0 .. L-2 as one kernel per image (attn_block.hip; tuning attn_fuse=1).
    // Measured slower than the three kernels (B/32 88.5-88.8k -> 81.6-82.1k img/s same box), so off
    bool attn_fuse = false;
    bool round_split = true;
    // tiles of the two launches (0 = the role's); tuning split_variants. r05: 72 as the main
    // launch measured +0.3-0.6 % with the bias as its first MFMA's C (profiles/r05/
    // b32_wb2_split72_ab.txt) and -0.3 % once its arithmetic was made v62's (bias in the epilogue,
    // so that the tile choice never changes a result; profiles/r05/final_defaults_vs_r04.txt)
    int split_main = 62, split_tail = 81;
    // c_fc with >= 2 whole rounds of 256x256 tiles plus a remainder: one balanced launch of
    // variant 75 instead of the round split (tuning fc_balanced; gemm() below)
    bool fc_balanced = true;
    int fc_bal_var = 75;  // its tile: 75 (256 x 256, 200 x 3 at B/32 bs 256) or 77 (320 x 256, 240 x 2); tuning fc_balanced_variant
    // XCD map of the main launch (tile_of_block; tuning split_xcd): 34 = the 1-D remap over a
    // column-group-major order with 2 N-groups, so each XCD group keeps half of W (2.4 MB of
    // c_fc's 4.7) in its 4 MB L2 across its M sweep. Measured: c_fc 0.875-0.879 -> 0.863-0.867
    // ms per forward, main-launch traffic 1.59x -> 1.38x of algorithmic
    int split_xcd = 34;
    // c_fc -> c_proj intermediate u in the 16-row blocked layout (common.h blk16_off): c_fc's
    // accumulator-layout stores become 256-B runs per quarter-wave instead of 16 scattered
    // 16-B pieces, and c_proj's A k-tiles become contiguous 2 KB runs
    bool u_blk = true;
    // the Linear weights also in the 16-row blocked layout (GemmArgs.blk_w), read by: 2 = every
    // launch whose tile reads it (default since r05; a row-split c_fc reads one copy in both of its
    // launches), 1 = the launches on the 32-deep-k-step tiles only (72 / 74), 0 = none (no
    // copies). tuning w_blocked. B/32 bs 256: 87.2-87.4k -> 88.0-88.6k img/s against 0 (QKV 0.578 ->
    // 0.565, c_proj 0.627 -> 0.610 ms per forward; same box, profiles/r05/b32_final_wblk_ab.txt)
    int w_blk = 2;
    // ln_2's output h (c_fc's A operand) in the 16-row blocked layout on the 24-bit-residual
    // forward, so the c_fc staging fetches 1 KB runs (128-B L2 requests) instead of 64-B row
    // pieces (tuning h_blocked: 2 = through an LDS transpose in the LN kernel, the default; 1 = the
    // LN kernel's lanes store 8 B each at blk16_off; 0 = row-major). Same box, 3 alternations:
    // B/32 bs 256 83.45-83.49k -> 83.76-84.14k img/s with 2 (c_fc 0.81 -> 0.784 ms per forward,
    // LayerNorm +0.018), 83.08-83.48k with 1 (profiles/r06/hblk_inmodel_ab.txt). QKV's h stays
    // row-major: its 240x256 tile measured the same either way (profiles/r06/hblk_v1_inmodel_ab.txt)
    int h_blk = 3;
    // patch embedding as blocked im2col (the pixel cast writes the GEMM's A in the 16-row blocked
    // layout) + the pipelined 160x128 tile on blocked A and W, instead of the implicit GEMM over
    // the cast pixels (tuning patch_im2col; only where a cast pass runs anyway)
    int patch_im2col = 1;
    // rows per wave of the add + LayerNorm after c_proj (ln_1 of the next block, 24-bit stream):
    // 1 (3,200 workgroups at B/32 bs 256) or 2 (1,600)
    int ln1_rows = 1;
    // QKV's A in the 16-row blocked layout too (blocks 1..L-1: ln_1 after c_proj writes it as
    // ln_2 does for c_fc, h_blocked's 8-row form; block 0's comes row-major from embed_ln)
    int qkv_blk = 1;
    // one-key-block attention (N <= 64: ViT-B/32) as a persistent loop on attn_persist workgroups
    // per CU, each prefetching its next (image, head) unit (attention_p_kernel); 0 = one
    // workgroup per unit (attention_v2)
    int attn_persist = 0;
    int use_hblk() const { return use_x24() && !lnfold ? h_blk : 0; }
    // test hook (tuning trace_gemm=1): every role GEMM launch of gemm() / gemm8() appends
    // {role, tile variant, M, flags} here (clipvit_gemm_log), so a test can assert which kernel
    // path a configuration reaches. Off in the product path.
    bool trace = false;
    std::mutex trace_mu;
    std::vector<int> trace_log;
    void log_launch(int role, int variant, int M, int flags) {
        if (!trace) return;
        std::lock_guard<std::mutex> lk(trace_mu);
        trace_log.insert(trace_log.end(), {role, variant, M, flags});
    }
};

// flags of a clipvit_gemm_log entry
enum { LOG_BLK_W = 1, LOG_MX8 = 2, LOG_BLK_A = 4, LOG_BLK_C = 8 };

static std::string L(int i, const char* leaf) {
    return "visual.transformer.resblocks." + std::to_string(i) + "." + leaf;
}

static void expected_tensors(const clipvit_handle* h,
                             std::vector<std::pair<std::string, std::vector<int64_t>>>& out) {
    const int64_t D = h->D, P = h->cfg.patch_size;
    out.push_back({"visual.conv1.weight", {D, 3, P, P}});
    out.push_back({"visual.class_embedding", {D}});
    out.push_back({"visual.positional_embedding", {h->N, D}});
    out.push_back({"visual.ln_pre.weight", {D}});
    out.push_back({"visual.ln_pre.bias", {D}});
    for (int i = 0; i < h->cfg.layers; ++i) {
        out.push_back({L(i, "ln_1.weight"), {D}});
        out.push_back({L(i, "ln_1.bias"), {D}});
        out.push_back({L(i, "attn.in_proj_weight"), {3 * D, D}});
        out.push_back({L(i, "attn.in_proj_bias"), {3 * D}});
        out.push_back({L(i, "attn.out_proj.weight"), {D, D}});
        out.push_back({L(i, "attn.out_proj.bias"), {D}});
        out.push_back({L(i, "ln_2.weight"), {D}});
        out.push_back({L(i, "ln_2.bias"), {D}});
        out.push_back({L(i, "mlp.c_fc.weight"), {4 * D, D}});
        out.push_back({L(i, "mlp.c_fc.bias"), {4 * D}});
        out.push_back({L(i, "mlp.c_proj.weight"), {D, 4 * D}});
        out.push_back({L(i, "mlp.c_proj.bias"), {D}});
    }
    out.push_back({"visual.ln_post.weight", {D}});
    out.push_back({"visual.ln_post.bias", {D}});
    out.push_back({"visual.proj", {D, (int64_t)h->E}});
}

static int free_ws(Workspace* w) {
    if (!w) return 0;
    for (auto& l : w->lane) {
        hipFree(l.x);
        hipFree(l.h);
        hipFree(l.qkv);
        hipFree(l.u);
        hipFree(l.f);
        hipFree(l.st);
        hipFree(l.q8);
        hipFree(l.x16);
        if (l.done) hipEventDestroy(l.done);
        if (l.stream) hipStreamDestroy(l.stream);
    }
    if (w->fork) hipEventDestroy(w->fork);
    delete w;
    return 0;
}

static int lane_cap(const clipvit_handle* h) {
    const int half = (h->cfg.max_batch + 1) / 2;
    return std::max(half, std::min(h->cfg.max_batch, h->split_min - 1));
}

static int alloc_ws(clipvit_handle* h, Workspace** out) {
    Workspace* w = new Workspace();
    hipError_t e = hipEventCreateWithFlags(&w->fork, hipEventDisableTiming);
    for (auto& l : w->lane) {
        l.cap = lane_cap(h);
        const size_t rows = ((size_t)l.cap * h->N + 15) / 16 * 16;  // u: whole 16-row blocks
        const size_t R = h->cfg.image_size;
        const size_t Rw = (R / h->cfg.patch_size) * ((h->cfg.patch_size + 7) / 8 * 8);  // padded pixel rows
        const size_t ubytes = std::max(rows * 4 * h->D * 2, (size_t)l.cap * 3 * R * Rw * 2);
        if (e == hipSuccess) e = hipMalloc(&l.x, rows * h->D * sizeof(float));
        if (e == hipSuccess) e = hipMalloc(&l.h, rows * h->D * 2);
        if (e == hipSuccess) e = hipMalloc(&l.qkv, rows * 3 * h->D * 2);
        if (e == hipSuccess) e = hipMalloc(&l.u, ubytes);
        if (e == hipSuccess) e = hipMalloc((void**)&l.f, (size_t)l.cap * h->E * sizeof(float));
        if (e == hipSuccess && h->lnfold) e = hipMalloc((void**)&l.st, rows * (h->D / 128) * sizeof(float2));
        if (e == hipSuccess && h->mx8) e = hipMalloc((void**)&l.q8, rows * h->D + rows * h->D / 32);
        if (e == hipSuccess && h->mx8) e = hipMalloc(&l.x16, rows * h->D * 2);
        else if (e == hipSuccess && h->use_x24()) e = hipMalloc(&l.x16, rows * h->D * 3);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&l.done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking);
    }
    if (e != hipSuccess) {
        free_ws(w);
        g_err = std::string("workspace allocation failed: ") + hipGetErrorString(e);
        return CLIPVIT_E_NOMEM;
    }
    *out = w;
    return 0;
}

// Take a free workspace (allocating one if every pooled workspace is busy). Every use of a
// lane's buffers is ordered after the previous one through the lane's `done` event.
// True when every lane's last recorded GPU work has finished (a call taking it will not wait).
static bool ws_idle(const Workspace* w) {
    for (const auto& l : w->lane)
        if (hipEventQuery(l.done) != hipSuccess) return false;
    return true;
}

// Take a workspace for one call. Preference: a free one whose previous GPU work is done; then,
// while the pool is below max_inflight, a new one — so calls issued on different streams
// (batches in flight, e.g. bench.py alternating two streams) do not serialise on one
// workspace's events; otherwise any free one (the call is ordered after its previous user
// through the lanes' `done` events). With every workspace held by a concurrent host call, a
// new one is allocated (the reference's ThreadPoolExecutor pattern).
static int acquire_ws(clipvit_handle* h, hipStream_t s, Workspace** out) {
    Workspace* w = nullptr;
    bool grow = false;
    {
        std::lock_guard<std::mutex> lk(h->mu);
        Workspace *same = nullptr, *lru = nullptr;
        for (auto* c : h->pool) {
            if (!c || c->used) continue;
            if (ws_idle(c)) {
                w = c;
                break;
            }
            if (c->last_stream == s && (!same || c->last_use > same->last_use)) same = c;
            if (!lru || c->last_use < lru->last_use) lru = c;
        }
        // busy on the GPU: the caller's own stream orders it for free; otherwise grow up to
        // max_inflight before waiting on another stream's work (least recently used)
        if (!w) w = same;
        if (!w && (int)h->pool.size() >= h->max_inflight) w = lru;
        if (w) w->used = true;
        else grow = true;
    }
    if (grow) {
        int rc = alloc_ws(h, &w);
        if (rc) return rc;
        w->used = true;
        std::lock_guard<std::mutex> lk(h->mu);
        h->pool.push_back(w);
    }
    {
        std::lock_guard<std::mutex> lk(h->mu);
        w->last_stream = s;
        w->last_use = ++h->calls;
    }
    *out = w;
    return 0;
}

static void release_ws(clipvit_handle* h, Workspace* w) {
    std::lock_guard<std::mutex> lk(h->mu);
    w->used = false;
}

enum Role { R_QKV = 0, R_OUT, R_FC, R_PROJ, R_PATCH };

// LayerNorm-fold operands of a GEMM (EPI_LNF*, EPI_RES_STATS; GemmArgs)
struct Fold {
    const float* s = nullptr;
    const float2* st_in = nullptr;
    float2* st_out = nullptr;
    void* C2 = nullptr;
    int np = 0;
    size_t x24_plane = 0;  // EPI_RES_STATS: C = the 24-bit residual planes (GemmArgs.x24_plane)
};

static int gemm(hipStream_t s, clipvit_handle* h, int epi, const void* A, const void* W,
                const float* bias, void* C, int M, int N, int K, int ldc, int role, const Fold& fo = Fold(),
                Lane* lane = nullptr, const void* Wb = nullptr, bool ablk = false) {
    GemmArgs a{};
    a.A = A; a.W = W; a.bias = bias; a.C = C;
    a.M = M; a.N = N; a.K = K; a.ldc = ldc;
    a.lnf_s = fo.s; a.st_in = fo.st_in; a.st_out = fo.st_out; a.C2 = fo.C2; a.np = fo.np;
    a.x24_plane = fo.x24_plane;
    a.patch_g2 = h->G2; a.patch_ntok = h->N;
    a.xcd_n = h->xcd[role];
    a.ncu = h->ncu;
    // every R_FC output / R_PROJ input is the lane's u; forced single-buffer tiles (1-3) cannot
    // address the blocked layout, so those keep u row-major for both roles
    auto blk_ok = [](int v) { return v >= 8; };
    const bool ublk = h->u_blk && (!h->var_forced || (blk_ok(h->var[R_FC]) && blk_ok(h->var[R_PROJ])));
    a.blk_c = ublk && role == R_FC;
    a.blk_a = (ublk && role == R_PROJ) || ablk;  // ablk: A = h in the blocked layout (use_hblk)
    int variant = h->var[role];
    auto launch = [&](const GemmArgs& g, int v) {
        const int rc = launch_gemm(s, h->dt, epi, g, v);
        if (rc == 0)
            h->log_launch(role, v, g.M, (g.blk_w ? LOG_BLK_W : 0) | (g.blk_a ? LOG_BLK_A : 0) | (g.blk_c ? LOG_BLK_C : 0));
        return rc;
    };
    // the blocked copy of W (w_blocked) for the launches whose tile reads it
    auto wsel = [&](GemmArgs& g, int v) {
        const bool blk = Wb && g.ksplit <= 1 &&
                         (h->w_blk == 2 ? v >= 8 : (h->w_blk == 1 && (v == 72 || v == 74)));
        g.W = blk ? Wb : W;
        g.blk_w = blk;
    };
    // Large-M shapes (L/14@336: M = 73,856; B/16): with several rounds of 256x256 tiles the
    // quantization loss that made the smaller tiles win at B/32 is gone and the 256x256 tile's
    // lower LDS fill per FLOP wins — measured: config 4 1,918 -> 2,072 img/s; B/16 c_fc (2,364
    // tiles) and out/c_proj (591 tiles, N = 768 roles from 2 rounds) 19.3k -> 20.2k img/s.
    // B/32's c_fc (600 tiles) takes the balanced v75 launch above instead.
    const long t256 = N % 256 == 0 ? (long)((M + 255) / 256) * (N / 256) : 0;
    // Whole-round row split (QKV / c_fc, 16-bit outputs). When the 256x256 tiles of a shape fill
    // R whole rounds of the CUs plus a remainder of at most half a round (B/32 c_fc at bs 128:
    // 300 tiles = 1 round + 44), rows [0, M1) — the most 256-row tiles that fit in R rounds,
    // 1-D block map so every XCD gets the same tile count — run on 256x256 tiles and rows
    // [M1, M) on the role's small tile as a second launch. Row-wise independent outputs:
    // bit-identical to one launch. Measured (c_fc 12800 x 3072 x 768): 81.6 us in one launch
    // (128x128) or 77.6 (256x256, 3 rounds) -> 54.3 + 15.9 = 70.2 us.
    // the main launch's tile width: every pipelined variant a round split can use is 256 wide
    // (8 / 62 / 72 / 74: 256x256, 98: 240x256)
    const int bn = 256;
    // (the ping-pong main tiles, split_main >= 60, have the 16-bit STORE / GELU epilogues only:
    // the LayerNorm-fold epilogues take the single-launch path below)
    const bool split_epi = epi == EPI_STORE || epi == EPI_GELU ||
                           ((epi == EPI_LNF || epi == EPI_LNF_GELU) && h->split_main < 60);
    if (h->round_split && !h->var_forced && (role == R_FC || role == R_QKV) && t256 &&
        N % bn == 0 && t256 < 4L * h->ncu && split_epi) {
        const long nN = N / bn, tm = (long)((M + 255) / 256) * nN;
        const long R = tm / h->ncu, rem = tm % h->ncu;
        const long m1 = R * h->ncu / nN * 256;
        if (role == R_FC && h->fc_balanced && R >= 2 && rem > 0 && epi == EPI_GELU) {
            // c_fc with >= 2 whole rounds + a remainder (B/32 bs 256: 600 tiles): one launch of
            // variant 75, the 32-deep-k-step tile on the fewest workgroups that keep ceil(tiles /
            // CUs) tiles each (200 x 3). Same arithmetic as the split (v62 + v81), so the same
            // bits; 69.4 against 71.9 us kernel-level, B/32 +0.7 % same box (3 alternations,
            // profiles/r05/balanced_grid_probe.txt)
            a.xcd_n = h->split_xcd;
            wsel(a, h->fc_bal_var);
            if (launch(a, h->fc_bal_var) == 0) return 0;
            wsel(a, 0);
            a.xcd_n = h->xcd[role];
        }
        if (R >= 1 && rem > 0 && 2 * rem <= h->ncu && m1 > 0 && m1 < M) {
            GemmArgs b = a;
            b.M = (int)m1;
            b.xcd_n = h->split_xcd;  // 1-D bijective remap (whole rounds per XCD group)
            if (h->split_main >= 60 && xcd_split_n(N / 256, b.xcd_n)) b.xcd_n = 0;  // ping-pong: 1-D maps only
            GemmArgs c = a;
            c.A = (const unsigned char*)A + (size_t)m1 * K * 2;
            c.C = (unsigned char*)C + (size_t)m1 * ldc * 2;
            if (c.st_in) c.st_in += (size_t)m1 * c.np;
            c.M = M - (int)m1;
            c.xcd_n = h->xcd[role];  // tail: the role's partition (main: 1-D, whole rounds per XCD)
            const int tv = h->split_tail ? h->split_tail : variant;
            wsel(b, h->split_main);
            wsel(c, tv);
            if (!b.blk_w) wsel(c, 0);  // both launches read one copy of W (the tail reuses the main's L2 lines)
            if (launch(b, h->split_main) == 0 && launch(c, tv) == 0)
                return 0;
            g_err = "gemm: round split failed M=" + std::to_string(M) + " N=" + std::to_string(N);
            return CLIPVIT_E_INVALID;
        }
    }
    // (c_fc's QuickGELU epilogue stores directly from the accumulators, v8: measured L/14@336
    // c_fc 7.79 -> 7.52 ms, B/16 1.59 -> 1.52 ms per lane-forward against the LDS-staged v80)
    if (!h->var_forced && role != R_PATCH &&
        (t256 >= 4L * h->ncu || ((role == R_OUT || role == R_PROJ) && t256 >= 2L * h->ncu))) {
        variant = 8;
        const int lv = role == R_QKV ? h->large_var[0] : role == R_FC ? h->large_var[1]
                     : role == R_OUT ? h->large_var[2] : role == R_PROJ ? h->large_var[3] : 0;
        if (lv && (epi == EPI_STORE || epi == EPI_GELU)) {
            a.xcd_n = lv / 100;
            variant = lv % 100;
        }
    }
    // a tuned variant that does not tile this shape (or, for the persistent tiles >= 60, lacks
    // the epilogue: the LayerNorm-fold ones) falls back to a pipelined tile, then the shape-based
    // choice
    wsel(a, variant);
    int rc = launch(a, variant);
    if (rc != 0 && variant >= 60) {
        const int fv = N % 256 == 0 ? 98 : 22;
        wsel(a, fv);
        rc = launch(a, fv);
    }
    wsel(a, 0);
    if (rc != 0 && launch(a, 0) != 0) {
        g_err = "gemm: unsupported shape M=" + std::to_string(M) + " N=" + std::to_string(N) +
                " K=" + std::to_string(K);
        return CLIPVIT_E_INVALID;
    }
    return 0;
}

// conv1 as an implicit GEMM over the pixels (gemm.hip PIMPL): 16-bit pixels of the compute type
// feed the patch tiles directly; other input dtypes are cast once into the u buffer.
static int patch_embed(clipvit_handle* h, hipStream_t s, const void* pix, int in_dtype, int B, Lane* w) {
    const int R = h->cfg.image_size, P = h->cfg.patch_size;
    if (h->patch_im2col && (P % 8 || in_dtype != h->dt) && h->Kp <= 4 * h->D) {
        // blocked im2col into u ([B G^2 rows padded to 16, Kp] <= u's [B N, 4 D]), then the
        // pipelined 160x128 tile (v22) on blocked A and W; same k order and k-tile sequence as
        // the implicit GEMM below
        if (launch_im2col_blk(s, in_dtype, h->dt, pix, w->u, B, R, P, h->Kp) != 0) {
            g_err = "patch embedding: unsupported patch size for im2col";
            return CLIPVIT_E_INVALID;
        }
        GemmArgs a{};
        a.A = w->u; a.W = h->wpatch_b; a.bias = nullptr; a.C = w->x;
        a.M = B * h->G2; a.N = h->D; a.K = h->Kp; a.ldc = h->D;
        a.patch_g2 = h->G2; a.patch_ntok = h->N;
        a.xcd_n = h->xcd[R_PATCH];
        a.blk_a = 1; a.blk_w = 1;
        if (launch_gemm(s, h->dt, EPI_PATCH, a, 22) != 0) {
            g_err = "patch embedding: explicit patch GEMM refused the shape";
            return CLIPVIT_E_INVALID;
        }
        return 0;
    }
    const void* px16 = pix;
    int Rw = R;
    if (P % 8) {  // P = 14: patch rows padded to 16 pixels (aligned 16-byte chunks)
        Rw = (R / P) * 16;
        launch_cast_pixels_padded(s, in_dtype, h->dt, pix, w->u, B, R, P);
        px16 = w->u;
    } else if (in_dtype != h->dt) {
        launch_cast_pixels(s, in_dtype, h->dt, pix, w->u, (size_t)B * 3 * R * R);
        px16 = w->u;
    }
    GemmArgs a{};
    a.A = px16; a.W = h->wpatch; a.bias = nullptr; a.C = w->x;
    a.M = B * h->G2; a.N = h->D; a.K = h->Kp; a.ldc = h->D;
    a.patch_g2 = h->G2; a.patch_ntok = h->N; a.patch_R = R; a.patch_Rw = Rw;
    a.xcd_n = h->xcd[R_PATCH];
    if (launch_patch_gemm(s, h->dt, P, a) != 0) {
        g_err = "patch embedding: unsupported patch size / width";
        return CLIPVIT_E_INVALID;
    }
    return 0;
}

// MX-fp8 GEMM: A = (A8, A8 + M*K scales), W = packed (N*K e4m3 bytes, then scales).
static int gemm8(hipStream_t s, clipvit_handle* h, int epi, const unsigned char* A8,
                 const void* Wq, const float* bias, void* C, int M, int N, int K, int ldc,
                 int role, bool ublk = false) {
    GemmArgs a{};
    // ublk: u8 (c_fc -> c_proj) in the 16-row blocked layout (blk8_off); its scales follow the
    // padded rows, since the last block's real rows spread over the whole block
    a.blk_c = ublk && role == R_FC;
    a.blk_a = ublk && role == R_PROJ;
    const size_t ma = a.blk_a ? (size_t)(M + 15) / 16 * 16 : (size_t)M;
    const size_t mc = a.blk_c ? (size_t)(M + 15) / 16 * 16 : (size_t)M;
    // blocked u8 scales ([K / 128][Mpad] dwords, GemmArgs.sc_rows) go with the blocked u8
    if (ublk && (role == R_FC || role == R_PROJ)) a.sc_rows = (int)((M + 15) / 16 * 16);
    a.A = A8; a.sA = A8 + ma * K;
    a.W = Wq; a.sW = (const unsigned char*)Wq + (size_t)N * K;
    a.bias = bias; a.C = C; a.M = M; a.N = N; a.K = K; a.ldc = ldc;
    if (epi == EPI_GELU_Q8) a.sC = (unsigned char*)C + mc * N;
    a.xcd_n = h->xcd[role];
    a.ncu = h->ncu;
    const int v8 = h->var8[role];
    auto launch = [&](const GemmArgs& g, int v) {
        const int rc = launch_gemm_mx8(s, CLIPVIT_BF16, epi, g, v);
        if (rc == 0) h->log_launch(role, v, g.M, LOG_MX8 | (g.blk_a ? LOG_BLK_A : 0) | (g.blk_c ? LOG_BLK_C : 0));
        return rc;
    };
    if ((v8 == 3 || v8 == 4) && xcd_split_n(N / 256, a.xcd_n)) a.xcd_n = 0;  // persistent MX tiles: 1-D maps
    // Whole-round row split of the MX c_fc (as gemm()'s for the 16-bit one): when the 256x256
    // tiles fill R whole rounds plus at most half a round (B/32 lane of 256 images: 600 tiles =
    // 2 rounds + 88), rows [0, M1) run on the persistent ping-pong and rows [M1, M) on the
    // 128x128 tile (two per CU) as a second launch. Row-wise independent: bit-identical to one
    // launch (same k order); the tail writes the same blocked u8 and its scales
    if (role == R_FC && epi == EPI_GELU_Q8 && v8 == 3 && h->round_split && h->mx8_split_tail && N % 256 == 0) {
        const long nN = N / 256, tm = (long)((M + 255) / 256) * nN;
        const long R = tm / h->ncu, rem = tm % h->ncu;
        const long m1 = R * h->ncu / nN * 256;
        if (R >= 1 && rem > 0 && 2 * rem <= h->ncu && m1 > 0 && m1 < M) {
            GemmArgs b = a, c = a;
            b.M = (int)m1;
            c.M = M - (int)m1;
            c.A = A8 + (size_t)m1 * K;
            c.sA = a.sA + (size_t)m1 * (K / 32);
            c.C = (unsigned char*)C + (size_t)m1 * ldc;  // = blk8_off(m1, 0, ldc): m1 % 16 == 0
            c.sC = a.sC + (a.sc_rows ? (size_t)m1 * 4 : (size_t)m1 * (ldc / 32));
            c.xcd_n = 0;
            if (launch(b, 3) == 0 && launch(c, h->mx8_split_tail) == 0)
                return 0;
            g_err = "gemm8: round split failed M=" + std::to_string(M) + " N=" + std::to_string(N);
            return CLIPVIT_E_INVALID;
        }
    }
    if (launch(a, v8) != 0 && launch(a, 0) != 0) {
        g_err = "gemm8: unsupported shape M=" + std::to_string(M) + " N=" + std::to_string(N) +
                " K=" + std::to_string(K);
        return CLIPVIT_E_INVALID;
    }
    return 0;
}

// Last block after its attention, on the class-token rows only (cls_prune): out_proj,
// LayerNorm, MLP and the residual adds are row-wise, and ln_post(x[:, 0, :]) @ proj reads only
// the class token, so the other B*(N-1) rows of this block are dead values. The CLS rows of x
// and of the attention output are gathered into compact [B, D] buffers carved from u (dead
// here); the arithmetic per row is the same kernels' (bit-identical result, tests/
// test_gpu_parity.py::test_cls_prune_is_bit_identical).
static int cls_tail(clipvit_handle* h, hipStream_t s, int B, Lane* w, float* f_out, Prof* prof,
                    const void* x16 = nullptr, bool x24 = false) {
    const int D = h->D, N = h->N;
    const LayerW& ly = h->layers[h->cfg.layers - 1];
    unsigned char* base = (unsigned char*)w->u;
    float* xc = (float*)base;
    u16* hc = (u16*)(base + (size_t)B * D * 4);
    u16* uc = hc + (size_t)B * D;
    // split-K partial products: the full-M qkv buffer is dead once gather_cls has run
    // (S * B * n * 4 bytes <= B * N * 3D * 2 bounds S per GEMM: 18 slices for c_fc at N = 50)
    float* part = (float*)w->qkv;
    launch_gather_cls(s, w->x, w->h, xc, hc, B, N, D, x16, x24);
    // M = B rows: 64x64 tiles alone give B/64 x N/64 workgroups whose K-long dependency chains
    // (48 k-tiles for c_proj) bound the tail, so each GEMM splits K into S slices (fixed per
    // shape: results do not depend on B) summed in slice order by the following kernel.
    // Measured tail 0.064 ms with one K chain (c_proj alone 27 us).
    auto g0 = [&](const void* A, const void* W, int n, int k, int& S) {
        S = 1;
        const int nkt = k / 64;
        const long cap = (long)N * 3 * D * 2 / ((long)n * 4);  // slices the dead qkv buffer holds
        for (int c = std::min(h->tail_smax, nkt); c >= 2; --c)
            if (nkt % c == 0 && k / c >= h->tail_kmin && c <= cap) { S = c; break; }
        GemmArgs a{};
        a.A = A; a.W = W; a.bias = nullptr; a.C = part;
        a.M = B; a.N = n; a.K = k; a.ldc = n; a.ksplit = S;
        if (launch_gemm(s, h->dt, EPI_F32, a, h->tail_var) != 0) {
            g_err = "cls tail gemm: unsupported shape";
            return CLIPVIT_E_INVALID;
        }
        return 0;
    };
    int rc, S;
    if ((rc = g0(hc, ly.wout, D, D, S))) return rc;
    if (prof) prof->mark(s, F_TAIL);
    launch_splitk_resid_ln(s, h->dt, xc, part, S, ly.bout, hc, ly.ln2g, ly.ln2b, B, D);
    if (prof) prof->mark(s, F_TAIL);
    if ((rc = g0(hc, ly.wfc, 4 * D, D, S))) return rc;
    launch_splitk_gelu(s, h->dt, part, S, ly.bfc, uc, B, 4 * D);
    if (prof) prof->mark(s, F_TAIL);
    if ((rc = g0(uc, ly.wproj, D, 4 * D, S))) return rc;
    launch_splitk_resid_ln(s, h->dt, xc, part, S, ly.bproj, nullptr, nullptr, nullptr, B, D);
    if (prof) prof->mark(s, F_TAIL);
    launch_cls_ln_proj(s, xc, h->lnpost_g, h->lnpost_b, h->proj, f_out, B, 1, D, h->E, h->head_cols);
    if (prof) prof->mark(s, F_HEAD);
    return 0;
}

// MX-fp8 encoder forward (same sequence as forward()). Blocks listed in
// mx8_skip run the 16-bit path; every LayerNorm writes the format its consumer block uses.
// resid16 (default): out_proj / c_proj store their bf16 branch outputs y, y2 in the dead qkv
// buffer and the deferred add + LayerNorm kernels do the fp32 residual adds, as in forward().
static int forward_mx8(clipvit_handle* h, hipStream_t s, const void* pix, int in_dtype, int B,
                       Lane* w, float* f_out, Prof* prof) {
    const int D = h->D, N = h->N, M = B * N;
    unsigned char* q8 = w->q8;
    unsigned char* q8s = q8 + (size_t)M * D;
    unsigned char* u8 = (unsigned char*)w->u;
    int rc;
    void* X16 = h->use_x16() ? w->x16 : nullptr;  // fp16 residual stream (nullptr: fp32 x)
    auto ln = [&](const float* g, const float* b, bool q) {
        if (q) launch_layernorm_q8(s, w->x, q8, q8s, g, b, M, D);
        else launch_layernorm(s, h->dt, w->x, w->h, g, b, M, D);
    };
    // x (+)= y (+ y2), then LayerNorm into the next GEMM's operand format. yb = y2: x = (x + y) + y2
    // stored; yb null: x + y, stored unless defer
    auto add_ln = [&](const void* ya, const void* yb, const float* g, const float* b, bool q, bool defer) {
        if (q) launch_add_layernorm_q8(s, w->x, ya, yb, q8, q8s, g, b, M, D, defer, X16);
        else if (yb || defer) launch_add_layernorm_deferred(s, h->dt, w->x, ya, yb, w->h, g, b, M, D, X16);
        else launch_add_layernorm(s, h->dt, w->x, ya, w->h, g, b, M, D, X16);
    };
    if (prof) prof->mark(s, F_EMBED);
    if ((rc = patch_embed(h, s, pix, in_dtype, B, w))) return rc;
    const LayerW& l0 = h->layers[0];
    if (h->q8_attn(0))
        launch_embed_ln_q8(s, w->x, q8, q8s, h->cls, h->pos, h->lnpre_g, h->lnpre_b, l0.ln1g,
                           l0.ln1b, B, N, D, X16);
    else
        launch_embed_ln(s, h->dt, w->x, w->h, h->cls, h->pos, h->lnpre_g, h->lnpre_b, l0.ln1g,
                        l0.ln1b, B, N, D, X16);
    if (prof) prof->mark(s, F_EMBED);
    void* y = w->qkv;
    void* y2 = (u16*)w->qkv + (size_t)M * D;
    for (int i = 0; i < h->cfg.layers; ++i) {
        const LayerW& ly = h->layers[i];
        // q: the attention roles (QKV, out_proj) in MX-fp8; qm: the MLP roles
        const bool q = h->q8_attn(i), qm = h->q8_mlp(i), last = i + 1 == h->cfg.layers;
        rc = q ? gemm8(s, h, EPI_STORE, q8, ly.wqkv, ly.bqkv, w->qkv, M, 3 * D, D, 3 * D, R_QKV)
               : gemm(s, h, EPI_STORE, w->h, ly.wqkv, ly.bqkv, w->qkv, M, 3 * D, D, 3 * D, R_QKV, Fold(), w, ly.wqkv_b);
        if (rc) return rc;
        if (prof) prof->mark(s, F_QKV);
        if (!q || !h->attn_q8 || launch_attention_q8(s, h->dt, w->qkv, q8, q8s, B, N, h->cfg.heads, h->attn_persist, h->ncu) != 0) {
            launch_attention(s, h->dt, w->qkv, w->h, B, N, h->cfg.heads, false, h->attn_persist, h->ncu);
            if (q) launch_quant_mx8(s, h->dt, w->h, q8, q8s, M, D);
        }
        if (prof) prof->mark(s, F_ATTN);
        if (last && h->cls_prune && !q && !qm) {  // bf16 last block: class-token rows only
            if ((rc = cls_tail(h, s, B, w, f_out, prof, X16))) return rc;
            HIPCHK(hipGetLastError());
            return 0;
        }
        const bool r16 = h->resid16, defer = r16 && h->defer_x && !last;
        const int eo = r16 ? EPI_STORE : EPI_RESID;
        void* co = r16 ? y : (void*)w->x;
        rc = q ? gemm8(s, h, eo, q8, ly.wout, ly.bout, co, M, D, D, D, R_OUT)
               : gemm(s, h, eo, w->h, ly.wout, ly.bout, co, M, D, D, D, R_OUT, Fold(), w, ly.wout_b);
        if (rc) return rc;
        if (prof) prof->mark(s, F_OUT);
        if (r16) add_ln(y, nullptr, ly.ln2g, ly.ln2b, qm, defer);
        else ln(ly.ln2g, ly.ln2b, qm);
        if (prof) prof->mark(s, F_LN);
        const bool p16 = r16 && !last;
        // blocked u8: both MLP GEMMs on the persistent MX tiles (c_fc 3 or 4), whose epilogues are STORE / GELU_Q8
        // (the fp32 residual c_proj runs on the other MX tiles: row-major u8)
        const bool ublk = h->u_blk && p16 && (h->var8[R_FC] == 3 || h->var8[R_FC] == 4) && h->var8[R_PROJ] == 3;
        rc = qm ? gemm8(s, h, EPI_GELU_Q8, q8, ly.wfc, ly.bfc, u8, M, 4 * D, D, 4 * D, R_FC, ublk)
               : gemm(s, h, EPI_GELU, w->h, ly.wfc, ly.bfc, w->u, M, 4 * D, D, 4 * D, R_FC, Fold(), w, ly.wfc_b);
        if (rc) return rc;
        if (prof) prof->mark(s, F_FC);
        const int ep = p16 ? EPI_STORE : EPI_RESID;
        void* cp = p16 ? (defer ? y2 : y) : (void*)w->x;
        rc = qm ? gemm8(s, h, ep, u8, ly.wproj, ly.bproj, cp, M, D, 4 * D, D, R_PROJ, ublk)
               : gemm(s, h, ep, w->u, ly.wproj, ly.bproj, cp, M, D, 4 * D, D, R_PROJ, Fold(), w, ly.wproj_b);
        if (rc) return rc;
        if (prof) prof->mark(s, F_PROJ);
        if (!last) {
            const LayerW& nx = h->layers[i + 1];
            if (p16) add_ln(y, defer ? y2 : nullptr, nx.ln1g, nx.ln1b, h->q8_attn(i + 1), false);
            else ln(nx.ln1g, nx.ln1b, h->q8_attn(i + 1));
            if (prof) prof->mark(s, F_LN);
        }
    }
    launch_cls_ln_proj(s, w->x, h->lnpost_g, h->lnpost_b, h->proj, f_out, B, N, D, h->E, h->head_cols);
    if (prof) prof->mark(s, F_HEAD);
    HIPCHK(hipGetLastError());
    return 0;
}

// Class-token tail of the last block on the LayerNorm-fold path (see cls_tail): the gathered
// CLS rows go through the same per-row arithmetic as the full block — out_proj on the full-M
// out_proj tile (160x128, EPI_RES_STATS: x += ., x16, the 128-column statistics in the same
// order), c_fc with the folded ln_2, c_proj (+x, fp32); then ln_post @ proj. On fp32 x the
// features equal the unpruned forward's bit for bit; on the 24-bit residual planes they do not
// (the tail keeps the CLS rows of x in fp32, where the full block would re-round them to 24 bits),
// and the fold's tests hold them to the oracle bar instead.
static int cls_tail_fold(clipvit_handle* h, hipStream_t s, int B, Lane* w, float* f_out, Prof* prof,
                         const void* x24 = nullptr) {
    const int D = h->D, N = h->N, np = D / 128;
    const LayerW& ly = h->layers[h->cfg.layers - 1];
    unsigned char* base = (unsigned char*)w->u;
    float* xc = (float*)base;
    u16* hc = (u16*)(base + (size_t)B * D * 4);
    u16* yc = hc + (size_t)B * D;
    u16* uc = yc + (size_t)B * D;
    float2* sc = (float2*)(uc + (size_t)B * 4 * D);
    launch_gather_cls(s, w->x, w->h, xc, hc, B, N, D, x24, x24 != nullptr);
    auto g0 = [&](int epi, int variant, const void* A, const void* W, const float* bias, void* C, int n, int k,
                  const Fold& fo) {
        GemmArgs a{};
        a.A = A; a.W = W; a.bias = bias; a.C = C;
        a.M = B; a.N = n; a.K = k; a.ldc = n;
        a.lnf_s = fo.s; a.st_in = fo.st_in; a.st_out = fo.st_out; a.C2 = fo.C2; a.np = fo.np;
        if (launch_gemm(s, h->dt, epi, a, variant) != 0) {
            g_err = "cls tail gemm: unsupported shape";
            return CLIPVIT_E_INVALID;
        }
        return 0;
    };
    int rc;
    Fold fo;
    fo.st_out = sc; fo.C2 = yc; fo.np = np;
    if ((rc = g0(EPI_RES_STATS, 82, hc, ly.wout, ly.bout, xc, D, D, fo))) return rc;
    if (prof) prof->mark(s, F_TAIL);
    Fold f2;
    f2.s = ly.s_fc; f2.st_in = sc; f2.np = np;
    if ((rc = g0(EPI_LNF_GELU, h->tail_var, yc, ly.wfc, ly.bf_fc, uc, 4 * D, D, f2))) return rc;
    if (prof) prof->mark(s, F_TAIL);
    if ((rc = g0(EPI_RESID, h->tail_var, uc, ly.wproj, ly.bproj, xc, D, 4 * D, Fold()))) return rc;
    if (prof) prof->mark(s, F_TAIL);
    launch_cls_ln_proj(s, xc, h->lnpost_g, h->lnpost_b, h->proj, f_out, B, 1, D, h->E, h->head_cols);
    if (prof) prof->mark(s, F_HEAD);
    return 0;
}

// Encoder forward with the LayerNorm fold. Buffers: x fp32 residual;
// x16 = 16-bit copy of x (the A operand of QKV in h, of c_fc in the dead qkv buffer); st = the
// per-row 128-column statistics of x. Per block:
//   QKV   = EPI_LNF(x16 (h), W_qkv diag(ln_1.g))        -> qkv        [ln_1 folded]
//   attn  (qkv)                                          -> h
//   out   = EPI_RES_STATS(h, W_out): x += ., x16 -> qkv[0, M*D), st
//   c_fc  = EPI_LNF_GELU(x16 (qkv), W_fc diag(ln_2.g))  -> u          [ln_2 folded]
//   c_proj= EPI_RES_STATS(u, W_proj): x += ., x16 -> h, st
static int forward_fold(clipvit_handle* h, hipStream_t s, const void* pix, int in_dtype, int B, Lane* w,
                        float* f_out, Prof* prof) {
    const int D = h->D, N = h->N, M = B * N, np = D / 128;
    int rc;
    if (prof) prof->mark(s, F_EMBED);
    if ((rc = patch_embed(h, s, pix, in_dtype, B, w))) return rc;
    // X24: the residual stream in 24-bit planes (w->x then only holds the patch GEMM's rows)
    void* X24 = h->use_x24() ? w->x16 : nullptr;
    const size_t plane = (size_t)M * D * 2;
    launch_embed_stats(s, h->dt, w->x, w->h, w->st, h->cls, h->pos, h->lnpre_g, h->lnpre_b, B, N, D, X24);
    if (prof) prof->mark(s, F_EMBED);
    void* x16b = w->qkv;  // x16 after out_proj (qkv is dead once attention has read it)
    const int nl = h->cfg.layers;
    for (int i = 0; i < nl; ++i) {
        const LayerW& ly = h->layers[i];
        Fold fq;
        fq.s = ly.s_qkv; fq.st_in = w->st; fq.np = np;
        if ((rc = gemm(s, h, EPI_LNF, w->h, ly.wqkv, ly.bf_qkv, w->qkv, M, 3 * D, D, 3 * D, R_QKV, fq))) return rc;
        if (prof) prof->mark(s, F_QKV);
        launch_attention(s, h->dt, w->qkv, w->h, B, N, h->cfg.heads, false, h->attn_persist, h->ncu);
        if (prof) prof->mark(s, F_ATTN);
        if (i + 1 == nl && h->cls_prune) {
            if ((rc = cls_tail_fold(h, s, B, w, f_out, prof, X24))) return rc;
            HIPCHK(hipGetLastError());
            return 0;
        }
        Fold fo;
        fo.st_out = w->st; fo.C2 = x16b; fo.np = np; fo.x24_plane = X24 ? plane : 0;
        void* xres = X24 ? X24 : (void*)w->x;
        if ((rc = gemm(s, h, EPI_RES_STATS, w->h, ly.wout, ly.bout, xres, M, D, D, D, R_OUT, fo))) return rc;
        if (prof) prof->mark(s, F_OUT);
        Fold ff;
        ff.s = ly.s_fc; ff.st_in = w->st; ff.np = np;
        if ((rc = gemm(s, h, EPI_LNF_GELU, x16b, ly.wfc, ly.bf_fc, w->u, M, 4 * D, D, 4 * D, R_FC, ff))) return rc;
        if (prof) prof->mark(s, F_FC);
        Fold fp;
        fp.st_out = w->st; fp.C2 = w->h; fp.np = np; fp.x24_plane = fo.x24_plane;
        if ((rc = gemm(s, h, EPI_RES_STATS, w->u, ly.wproj, ly.bproj, xres, M, D, 4 * D, D, R_PROJ, fp))) return rc;
        if (prof) prof->mark(s, F_PROJ);
    }
    launch_cls_ln_proj(s, w->x, h->lnpost_g, h->lnpost_b, h->proj, f_out, B, N, D, h->E, h->head_cols);
    if (prof) prof->mark(s, F_HEAD);
    HIPCHK(hipGetLastError());
    return 0;
}

// Encoder forward for B images on stream s with lane buffers w; writes the projected
// (un-normalised) features to f_out.
static int forward(clipvit_handle* h, hipStream_t s, const void* pix, int in_dtype, int B,
                   Lane* w, float* f_out, Prof* prof) {
    if (h->mx8) return forward_mx8(h, s, pix, in_dtype, B, w, f_out, prof);
    if (h->lnfold) return forward_fold(h, s, pix, in_dtype, B, w, f_out, prof);
    const int D = h->D, N = h->N, M = B * N;
    int rc;
    if (prof) prof->mark(s, F_EMBED);
    if ((rc = patch_embed(h, s, pix, in_dtype, B, w))) return rc;
    const LayerW& l0 = h->layers[0];
    // X24: the residual stream in 24-bit planes (w->x then only holds the patch GEMM's rows)
    void* X24 = h->use_x24() ? w->x16 : nullptr;
    const int hb = h->use_hblk();
    const bool hq = hb != 0 && h->qkv_blk;  // blocked h for QKV (blocks >= 1)
    launch_embed_ln(s, h->dt, w->x, w->h, h->cls, h->pos, h->lnpre_g, h->lnpre_b, l0.ln1g, l0.ln1b,
                    B, N, D, X24, X24 != nullptr);
    if (prof) prof->mark(s, F_EMBED);
    // 16-bit residual branch outputs (resid16) reuse the qkv buffer: qkv is dead once attention
    // has read it. y = out_proj's branch, y2 = c_proj's. With deferred adds (defer_x), the add
    // after out_proj only feeds ln_2 (x is not written back) and the add after c_proj computes
    // (x + y) + y2 — the same fp32 additions in the same order — and stores x once per block.
    void* y = w->qkv;
    void* y2 = (u16*)w->qkv + (size_t)M * D;
    const int nl = h->cfg.layers;
    for (int i = 0; i < nl; ++i) {
        const LayerW& ly = h->layers[i];
        const bool last = i + 1 == nl;
        if ((rc = gemm(s, h, EPI_STORE, w->h, ly.wqkv, ly.bqkv, w->qkv, M, 3 * D, D, 3 * D, R_QKV, Fold(), w, ly.wqkv_b,
                       hq && i > 0)))
            return rc;
        if (prof) prof->mark(s, F_QKV);
        const bool defer = h->resid16 && h->defer_x && !last;
        // blocks 0 .. L-2 of ViT-B/32: attention, out_proj, x += y and ln_2 in one kernel per image
        // (x then already holds x + y, so the ln_1 below adds only c_proj's y2)
        const bool fused = h->attn_fuse && defer && X24 && hb != 0 &&
                           launch_attn_out_ln(s, h->dt, w->qkv, ly.wout_b, ly.bout, X24, (size_t)M * D * 2, ly.ln2g,
                                              ly.ln2b, w->h, B, N, D) == 0;
        if (!fused) launch_attention(s, h->dt, w->qkv, w->h, B, N, h->cfg.heads, false, h->attn_persist, h->ncu);
        if (prof) prof->mark(s, F_ATTN);
        if (last && h->cls_prune) {
            if ((rc = cls_tail(h, s, B, w, f_out, prof, X24, X24 != nullptr))) return rc;
            HIPCHK(hipGetLastError());
            return 0;
        }
        if (fused) {
        } else if (h->resid16) {
            if ((rc = gemm(s, h, EPI_STORE, w->h, ly.wout, ly.bout, y, M, D, D, D, R_OUT, Fold(), w, ly.wout_b))) return rc;
            if (prof) prof->mark(s, F_OUT);
            if (defer) launch_add_layernorm_deferred(s, h->dt, w->x, y, nullptr, w->h, ly.ln2g, ly.ln2b, M, D, X24, X24 != nullptr, hb);
            else launch_add_layernorm(s, h->dt, w->x, y, w->h, ly.ln2g, ly.ln2b, M, D);
        } else {
            if ((rc = gemm(s, h, EPI_RESID, w->h, ly.wout, ly.bout, w->x, M, D, D, D, R_OUT))) return rc;
            if (prof) prof->mark(s, F_OUT);
            launch_layernorm(s, h->dt, w->x, w->h, ly.ln2g, ly.ln2b, M, D);
        }
        if (prof) prof->mark(s, F_LN);
        if ((rc = gemm(s, h, EPI_GELU, w->h, ly.wfc, ly.bfc, w->u, M, 4 * D, D, 4 * D, R_FC, Fold(), w, ly.wfc_b, hb != 0)))
            return rc;
        if (prof) prof->mark(s, F_FC);
        if (h->resid16 && !last) {
            void* yo = defer ? y2 : y;
            if ((rc = gemm(s, h, EPI_STORE, w->u, ly.wproj, ly.bproj, yo, M, D, 4 * D, D, R_PROJ, Fold(), w, ly.wproj_b)))
                return rc;
            if (prof) prof->mark(s, F_PROJ);
            const LayerW& nx = h->layers[i + 1];
            if (fused) launch_add_layernorm_x24_store(s, h->dt, X24, y2, w->h, nx.ln1g, nx.ln1b, M, D, hq ? 3 : 0);
            else if (defer) launch_add_layernorm_deferred(s, h->dt, w->x, y, y2, w->h, nx.ln1g, nx.ln1b, M, D, X24, X24 != nullptr,
                                                          hq ? 3 : X24 && h->ln1_rows == 2 ? 4 : 0);
            else launch_add_layernorm(s, h->dt, w->x, y, w->h, nx.ln1g, nx.ln1b, M, D);
            if (prof) prof->mark(s, F_LN);
        } else {
            if ((rc = gemm(s, h, EPI_RESID, w->u, ly.wproj, ly.bproj, w->x, M, D, 4 * D, D, R_PROJ)))
                return rc;
            if (prof) prof->mark(s, F_PROJ);
            if (!last) {
                launch_layernorm(s, h->dt, w->x, w->h, h->layers[i + 1].ln1g, h->layers[i + 1].ln1b, M, D);
                if (prof) prof->mark(s, F_LN);
            }
        }
    }
    launch_cls_ln_proj(s, w->x, h->lnpost_g, h->lnpost_b, h->proj, f_out, B, N, D, h->E, h->head_cols);
    if (prof) prof->mark(s, F_HEAD);
    HIPCHK(hipGetLastError());
    return 0;
}

static size_t pixel_bytes(const clipvit_handle* h, int dtype) {
    const size_t R = h->cfg.image_size;
    return 3 * R * R * (dtype == CLIPVIT_F32 ? 4 : 2);
}

static int lane_batch(const clipvit_handle* h, int B) {
    return B >= h->split_min ? (B + 1) / 2 : B;
}

// Run body(stream, lane, first_image, count) for the whole batch: split over the two lane
// streams (fork/join with the caller's stream s by events) when B >= SPLIT_MIN, otherwise on
// s itself with lane 0. Lane buffers are always ordered after their previous user.
template <typename F>
static int run_lanes(clipvit_handle* h, hipStream_t s, int B, Workspace* w, F&& body) {
    if (B < h->split_min) {
        Lane& l = w->lane[0];
        HIPCHK(hipStreamWaitEvent(s, l.done, 0));
        const int rc = body(s, &l, 0, B);
        HIPCHK(hipEventRecord(l.done, s));
        return rc;
    }
    HIPCHK(hipEventRecord(w->fork, s));
    const int b0 = (B + 1) / 2;
    int rc = 0;
    for (int i = 0; i < kLanes; ++i) {
        Lane& l = w->lane[i];
        const int off = i == 0 ? 0 : b0, cnt = i == 0 ? b0 : B - b0;
        HIPCHK(hipStreamWaitEvent(l.stream, w->fork, 0));
        HIPCHK(hipStreamWaitEvent(l.stream, l.done, 0));
        if (!rc) rc = body(l.stream, &l, off, cnt);
        HIPCHK(hipEventRecord(l.done, l.stream));
        HIPCHK(hipStreamWaitEvent(s, l.done, 0));
    }
    (void)h;
    return rc;
}

static int check_call(clipvit_handle* h, const void* pix, int dtype, int B) {
    if (!h) FAIL(CLIPVIT_E_INVALID, "null handle");
    if (!h->loaded) FAIL(CLIPVIT_E_STATE, "weights not loaded");
    if (!pix) FAIL(CLIPVIT_E_INVALID, "null pixel buffer");
    if (dtype < 0 || dtype > 2) FAIL(CLIPVIT_E_INVALID, "bad pixel dtype");
    if (B <= 0 || B > h->cfg.max_batch)
        FAIL(CLIPVIT_E_INVALID, "batch " + std::to_string(B) + " outside [1, max_batch=" +
                                    std::to_string(h->cfg.max_batch) + "]");
    return 0;
}

// Re-pack every Linear from its fp32 master (optionally with merged LoRA deltas).
static int pack_linear(clipvit_handle* h, hipStream_t s, const std::string& name, void* dst,
                       const float* src) {
    const auto& sh = h->shapes[name];
    const int N = (int)sh[0];
    int K = 1;
    for (size_t i = 1; i < sh.size(); ++i) K *= (int)sh[i];
    const int Kp = (K + 63) / 64 * 64;
    const float* w = src ? src : h->master[name];
    int layer = -1;
    const std::string pre = "visual.transformer.resblocks.";
    if (name.compare(0, pre.size(), pre) == 0) layer = atoi(name.c_str() + pre.size());
    const bool mlp_role = name.find(".mlp.") != std::string::npos;
    if (layer >= 0 && (mlp_role ? h->q8_mlp(layer) : h->q8_attn(layer))) {
        if (K % 128) FAIL(CLIPVIT_E_INVALID, "MX-fp8 Linear needs in_features % 128 == 0: " + name);
        unsigned char* q = (unsigned char*)dst;
        launch_pack_weight_mx8(s, w, q, q + (size_t)N * K, N, K, K);
        return 0;
    }
    // LayerNorm fold: in_proj carries ln_1, c_fc carries ln_2 (W' = W diag(gamma), s_n, b'_n)
    if (h->lnfold && layer >= 0) {
        const bool qkv = name.find("attn.in_proj_weight") != std::string::npos;
        const bool fc = name.find("mlp.c_fc.weight") != std::string::npos;
        if (qkv || fc) {
            LayerW& ly = h->layers[layer];
            const float* g = qkv ? ly.ln1g : ly.ln2g;
            const float* be = qkv ? ly.ln1b : ly.ln2b;
            const float* b = qkv ? ly.bqkv : ly.bfc;
            launch_lnfold_prep(s, h->dt, w, g, be, b, h->scratch2, qkv ? ly.s_qkv : ly.s_fc,
                               qkv ? ly.bf_qkv : ly.bf_fc, N, K);
            launch_pack_weight(s, h->dt, h->scratch2, dst, N, K, Kp);
            return 0;
        }
    }
    launch_pack_weight(s, h->dt, w, dst, N, K, Kp);
    if (layer >= 0) {  // the blocked copy (w_blocked) follows every re-pack (LoRA merges too)
        const LayerW& ly = h->layers[layer];
        void* blk = dst == ly.wqkv ? ly.wqkv_b : dst == ly.wfc ? ly.wfc_b : dst == ly.wout ? ly.wout_b
                  : dst == ly.wproj ? ly.wproj_b : nullptr;
        if (blk) launch_blk16_relayout(s, dst, blk, N, Kp);
    }
    return 0;
}

extern "C" {

const char* clipvit_last_error(void) { return g_err.c_str(); }
int clipvit_abi_version(void) { return CLIPVIT_ABI_VERSION; }

int clipvit_create(const clipvit_config* cfg, int device, clipvit_handle** out) {
    g_err.clear();
    if (!cfg || !out) FAIL(CLIPVIT_E_INVALID, "null argument");
    const clipvit_config& c = *cfg;
    if (c.patch_size != 14 && c.patch_size != 16 && c.patch_size != 32)
        FAIL(CLIPVIT_E_INVALID, "patch_size must be 14, 16 or 32");
    if (c.image_size % c.patch_size) FAIL(CLIPVIT_E_INVALID, "image_size must be a multiple of patch_size");
    if (c.width % 256 || c.width < 512 || c.width > 1280)
        FAIL(CLIPVIT_E_INVALID, "width must be a multiple of 256 in [512, 1280]");
    if (c.heads * 64 != c.width) FAIL(CLIPVIT_E_INVALID, "heads * 64 must equal width");
    if (c.embed_dim % 128 || c.embed_dim <= 0 || c.embed_dim > 1280)
        FAIL(CLIPVIT_E_INVALID, "embed_dim must be a multiple of 128 in [128, 1280]");
    if (c.compute_dtype != CLIPVIT_BF16 && c.compute_dtype != CLIPVIT_F16 && c.compute_dtype != CLIPVIT_MXFP8)
        FAIL(CLIPVIT_E_INVALID, "compute_dtype must be BF16, F16 or MXFP8");
    if (c.layers <= 0 || c.max_batch <= 0) FAIL(CLIPVIT_E_INVALID, "layers/max_batch must be > 0");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) FAIL(CLIPVIT_E_INVALID, "bad device index");
    DeviceGuard dg(device);
    auto* h = new clipvit_handle();
    h->cfg = c;
    h->device = device;
    h->G = c.image_size / c.patch_size;
    h->G2 = h->G * h->G;
    h->N = h->G2 + 1;
    h->D = c.width;
    h->E = c.embed_dim;
    // patch length in the implicit patch GEMM's k order (row length padded to a multiple of 8)
    h->K3 = 3 * c.patch_size * ((c.patch_size + 7) / 8 * 8);
    h->Kp = (h->K3 + 63) / 64 * 64;
    h->mx8 = c.compute_dtype == CLIPVIT_MXFP8;
    h->dt = h->mx8 ? CLIPVIT_BF16 : c.compute_dtype;  // 16-bit type of everything not MX-fp8
    // 16-bit residual branch outputs for both 16-bit types (bf16 too since r02: measured 76.3k ->
    // 78.9k img/s at bs 256 with the logit error unchanged, 4.35e-3 -> 4.13e-3)
    h->resid16 = true;  // fp16, bf16 and MX-fp8 (its bf16 branch outputs)
    // off by default: measured slower (the residual epilogues run in lockstep
    // at the end of one-round GEMMs; B/32 78.2k -> 74.3k img/s, B/16 20.6k -> 19.2k, L/14 2116 -> 2008)
    h->lnfold = false;
    h->split_min = std::max(SPLIT_IMAGES, (SPLIT_TOKENS + h->N - 1) / h->N);
    // default bf16 blocks: the MLP of the first two and last two blocks, the attention roles of
    // block 1 and the last block only (the last block runs the class-token tail). Measured on
    // three image / text seeds against the bf16 engine at CLIP logit scale: 1.79e-2 (bar 2e-2;
    // 1.93e-2 with the attention roles of all four blocks in bf16, 2.04e-2 with block 11's only)
    // and config 5 +1.7 % (tools/mx_skip_sweep.py)
    if (h->mx8) {
        const int L = c.layers;
        for (int b : {0, 1, L - 2, L - 1})
            if (b >= 0 && b < 64) h->mx8_skip_mlp |= 1ull << b;
        for (int b : {1, L - 1})
            if (b >= 0 && b < 64) h->mx8_skip |= 1ull << b;
    }
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
            h->ncu = ncu;
    }
    *out = h;
    return 0;
}

// ---- clipvit_set_tuning: the measured alternatives of DESIGN.md, for tests and A/B tools only ----
static bool parse_int(const std::string& v, int& out) {
    char* e = nullptr;
    const long x = strtol(v.c_str(), &e, 10);
    if (v.empty() || !e || *e) return false;
    out = (int)x;
    return true;
}
// "a,b,c" -> up to n ints; every field must parse
static bool parse_list(const std::string& v, int* out, int n) {
    size_t pos = 0;
    for (int k = 0; k < n && pos <= v.size(); ++k) {
        const size_t q = v.find(',', pos);
        if (!parse_int(v.substr(pos, q == std::string::npos ? std::string::npos : q - pos), out[k])) return false;
        if (q == std::string::npos) return true;
        pos = q + 1;
    }
    return pos > v.size();
}
// "i,j,..." -> bit mask of block indices ("" = none)
static bool parse_mask(const std::string& v, uint64_t& m) {
    m = 0;
    size_t pos = 0;
    while (pos < v.size()) {
        const size_t q = v.find(',', pos);
        int b = 0;
        if (!parse_int(v.substr(pos, q == std::string::npos ? std::string::npos : q - pos), b) || b < 0 || b >= 64)
            return false;
        m |= 1ull << b;
        if (q == std::string::npos) break;
        pos = q + 1;
    }
    return true;
}

static int apply_tuning(clipvit_handle* h, const std::string& k, const std::string& v) {
    int x = 0;
    auto flag = [&](bool& dst) {
        if (!parse_int(v, x)) return false;
        dst = x != 0;
        return true;
    };
    bool ok = true;
    if (k == "resid16") ok = flag(h->resid16);
    else if (k == "defer_x") ok = flag(h->defer_x);
    else if (k == "lnfold") ok = flag(h->lnfold);  // resolved after every key (clipvit_set_tuning)
    else if (k == "cls_prune") ok = flag(h->cls_prune);
    else if (k == "round_split") ok = flag(h->round_split);
    else if (k == "fc_balanced") ok = flag(h->fc_balanced);
    else if (k == "fc_balanced_variant") ok = parse_int(v, h->fc_bal_var) && (h->fc_bal_var == 75 || h->fc_bal_var == 77);
    else if (k == "attn_q8") ok = flag(h->attn_q8);
    else if (k == "attn_fuse") ok = flag(h->attn_fuse);
    else if (k == "x16") ok = flag(h->x16);
    else if (k == "x24") ok = flag(h->x24);
    else if (k == "u_blocked") ok = flag(h->u_blk);
    else if (k == "trace_gemm") ok = flag(h->trace);
    else if (k == "h_blocked") ok = parse_int(v, h->h_blk) && h->h_blk >= 0 && h->h_blk <= 3;
    else if (k == "patch_im2col") ok = parse_int(v, h->patch_im2col) && (h->patch_im2col == 0 || h->patch_im2col == 1);
    else if (k == "qkv_blk") ok = parse_int(v, h->qkv_blk) && (h->qkv_blk == 0 || h->qkv_blk == 1);
    else if (k == "ln1_rows") ok = parse_int(v, h->ln1_rows) && (h->ln1_rows == 1 || h->ln1_rows == 2);
    else if (k == "attn_persist") ok = parse_int(v, h->attn_persist) && h->attn_persist >= 0 && h->attn_persist <= 4;
    else if (k == "w_blocked") ok = parse_int(v, h->w_blk) && h->w_blk >= 0 && h->w_blk <= 2;
    else if (k == "split_variants") {  // "main[,tail]": main a 256x256 tile (8, 62, 72, 74)
        int m[2] = {h->split_main, h->split_tail};
        ok = parse_list(v, m, 2) && (m[0] == 8 || m[0] == 62 || m[0] == 72 || m[0] == 74);
        if (ok) { h->split_main = m[0]; h->split_tail = m[1]; }
    } else if (k == "tail_variant") ok = parse_int(v, h->tail_var);
    else if (k == "tail_kmin") ok = parse_int(v, h->tail_kmin) && h->tail_kmin >= 64 && h->tail_kmin % 64 == 0;
    else if (k == "head_cols") ok = parse_int(v, h->head_cols) && (h->head_cols == 64 || h->head_cols == 32);
    else if (k == "tail_smax") ok = parse_int(v, h->tail_smax) && h->tail_smax >= 1 && h->tail_smax <= 48;
    else if (k == "split_xcd") ok = parse_int(v, h->split_xcd);
    else if (k == "max_inflight") {
        ok = parse_int(v, x) && x >= 1;
        if (ok) h->max_inflight = x;
    } else if (k == "split_min") {  // <= 0: never split
        ok = parse_int(v, x);
        if (ok) h->split_min = x <= 0 ? SPLIT_NEVER : x;
    } else if (k == "gemm_xcd") ok = parse_list(v, h->xcd, 5);
    else if (k == "qkv_variant" || k == "fc_variant" || k == "out_variant" || k == "proj_variant") {
        // 100 * XCD map + tile of one role, the shape rules kept (gemm_variants forces all)
        ok = parse_int(v, x) && x > 0;
        const int r = k == "qkv_variant" ? R_QKV : k == "fc_variant" ? R_FC : k == "out_variant" ? R_OUT : R_PROJ;
        if (ok) {
            h->var[r] = x % 100;
            h->xcd[r] = x / 100;
        }
    }
    else if (k == "mx8_skip") {  // both masks
        ok = parse_mask(v, h->mx8_skip);
        if (ok) h->mx8_skip_mlp = h->mx8_skip;
    } else if (k == "mx8_skip_mlp") ok = parse_mask(v, h->mx8_skip_mlp);
    else if (k == "mx8_variants") ok = parse_list(v, h->var8, 4);
    else if (k == "mx8_split_tail") ok = parse_int(v, h->mx8_split_tail) && (h->mx8_split_tail == 0 || h->mx8_split_tail == 2 || h->mx8_split_tail == 5);
    else if (k == "large_variants") ok = parse_list(v, h->large_var, 4);
    else if (k == "gemm_variants") {
        ok = parse_list(v, h->var, 5);
        h->var_forced = ok;
    } else FAIL(CLIPVIT_E_INVALID, "unknown tuning key '" + k + "'");
    if (!ok) FAIL(CLIPVIT_E_INVALID, "bad tuning value " + k + "=" + v);
    return 0;
}

int clipvit_set_tuning(clipvit_handle* h, const char* spec) {
    g_err.clear();
    if (!h || !spec) FAIL(CLIPVIT_E_INVALID, "null argument");
    if (h->loaded || !h->pool.empty()) FAIL(CLIPVIT_E_STATE, "tuning must precede clipvit_load_weights");
    const std::string all(spec);
    struct KV { std::string k, v; };
    std::vector<KV> kv;
    size_t pos = 0;
    while (pos < all.size()) {
        size_t q = all.find(';', pos);
        if (q == std::string::npos) q = all.size();
        const std::string item = all.substr(pos, q - pos);
        pos = q + 1;
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        if (eq == std::string::npos) FAIL(CLIPVIT_E_INVALID, "tuning item without '=': " + item);
        kv.push_back({item.substr(0, eq), item.substr(eq + 1)});
    }
    // a bad item leaves the handle as it was: apply to a snapshot of the tunable fields first
    struct Tun {
        bool resid16, defer_x, lnfold, cls_prune, round_split, attn_q8, x16, x24, var_forced, u_blk, fc_balanced, trace, attn_fuse;
        int h_blk, patch_im2col, ln1_rows, qkv_blk, attn_persist, w_blk, fc_bal_var, split_main, split_tail, tail_var, tail_kmin, tail_smax, head_cols, split_xcd, max_inflight, split_min, mx8_split_tail;
        int xcd[5], var8[4], large_var[4], var[5];
        uint64_t mx8_skip, mx8_skip_mlp;
    };
    auto save = [](const clipvit_handle* g) {
        Tun t{g->resid16, g->defer_x, g->lnfold, g->cls_prune, g->round_split, g->attn_q8, g->x16, g->x24,
              g->var_forced, g->u_blk, g->fc_balanced, g->trace, g->attn_fuse, g->h_blk, g->patch_im2col, g->ln1_rows, g->qkv_blk, g->attn_persist, g->w_blk, g->fc_bal_var, g->split_main, g->split_tail, g->tail_var, g->tail_kmin, g->tail_smax, g->head_cols,
              g->split_xcd, g->max_inflight,
              g->split_min, g->mx8_split_tail, {}, {}, {}, {}, g->mx8_skip, g->mx8_skip_mlp};
        memcpy(t.xcd, g->xcd, sizeof t.xcd);
        memcpy(t.var8, g->var8, sizeof t.var8);
        memcpy(t.large_var, g->large_var, sizeof t.large_var);
        memcpy(t.var, g->var, sizeof t.var);
        return t;
    };
    const Tun before = save(h);
    for (const auto& e : kv) {
        const int rc = apply_tuning(h, e.k, e.v);
        if (rc) {
            h->resid16 = before.resid16; h->defer_x = before.defer_x; h->lnfold = before.lnfold;
            h->cls_prune = before.cls_prune; h->round_split = before.round_split; h->attn_q8 = before.attn_q8;
            h->x16 = before.x16; h->x24 = before.x24; h->var_forced = before.var_forced; h->u_blk = before.u_blk;
            h->fc_balanced = before.fc_balanced; h->trace = before.trace; h->attn_fuse = before.attn_fuse; h->h_blk = before.h_blk; h->patch_im2col = before.patch_im2col; h->ln1_rows = before.ln1_rows; h->qkv_blk = before.qkv_blk; h->attn_persist = before.attn_persist; h->w_blk = before.w_blk; h->fc_bal_var = before.fc_bal_var;
            h->split_main = before.split_main; h->split_tail = before.split_tail; h->tail_var = before.tail_var;
            h->tail_kmin = before.tail_kmin; h->tail_smax = before.tail_smax; h->head_cols = before.head_cols;
            h->split_xcd = before.split_xcd; h->max_inflight = before.max_inflight; h->split_min = before.split_min;
            h->mx8_split_tail = before.mx8_split_tail;
            memcpy(h->xcd, before.xcd, sizeof before.xcd);
            memcpy(h->var8, before.var8, sizeof before.var8);
            memcpy(h->large_var, before.large_var, sizeof before.large_var);
            memcpy(h->var, before.var, sizeof before.var);
            h->mx8_skip = before.mx8_skip;
            h->mx8_skip_mlp = before.mx8_skip_mlp;
            return rc;
        }
    }
    // the fold is fp16-only on the 16-bit branch path, D <= 1024 (<= 8 statistics groups per
    // row); resolved once after every key so that the spec's key order does not matter
    h->lnfold = h->lnfold && h->resid16 && h->dt == CLIPVIT_F16 && h->D <= 1024;
    return 0;
}

int clipvit_load_weights(clipvit_handle* h, const clipvit_tensor* tensors, size_t n) {
    g_err.clear();
    if (!h || (!tensors && n)) FAIL(CLIPVIT_E_INVALID, "null argument");
    DeviceGuard dg(h->device);
    std::unordered_map<std::string, const clipvit_tensor*> byname;
    for (size_t i = 0; i < n; ++i)
        if (tensors[i].name) byname[tensors[i].name] = &tensors[i];
    std::vector<std::pair<std::string, std::vector<int64_t>>> exp;
    expected_tensors(h, exp);
    // validate everything before touching the device
    for (auto& e : exp) {
        auto it = byname.find(e.first);
        if (it == byname.end()) FAIL(CLIPVIT_E_INVALID, "missing tensor " + e.first);
        const clipvit_tensor* t = it->second;
        bool ok = t->ndim == (int)e.second.size() && t->data;
        for (int d = 0; ok && d < t->ndim; ++d) ok = t->shape[d] == e.second[d];
        if (!ok) FAIL(CLIPVIT_E_INVALID, "bad shape/data for " + e.first);
    }
    for (auto& e : exp) {
        const clipvit_tensor* t = byname[e.first];
        size_t cnt = 1;
        for (auto d : e.second) cnt *= (size_t)d;
        float*& dst = h->master[e.first];
        if (!dst) HIPCHK(hipMalloc(&dst, cnt * sizeof(float)));
        HIPCHK(hipMemcpy(dst, t->data, cnt * sizeof(float), hipMemcpyHostToDevice));
        h->shapes[e.first] = e.second;
    }
    h->cls = h->master["visual.class_embedding"];
    h->pos = h->master["visual.positional_embedding"];
    h->lnpre_g = h->master["visual.ln_pre.weight"];
    h->lnpre_b = h->master["visual.ln_pre.bias"];
    h->lnpost_g = h->master["visual.ln_post.weight"];
    h->lnpost_b = h->master["visual.ln_post.bias"];
    h->proj = h->master["visual.proj"];
    // packed operands
    const size_t D = h->D;
    auto alloc16 = [&](void*& p, size_t elems) -> hipError_t {
        if (p) return hipSuccess;
        return hipMalloc(&p, elems * 2);
    };
    HIPCHK(alloc16(h->wpatch, D * h->Kp));
    HIPCHK(alloc16(h->wpatch_b, D * h->Kp));
    h->layers.resize(h->cfg.layers);
    size_t maxw = D * h->K3;
    // blocked weight copies of the Linears that pack_linear re-lays out: not for the MX-fp8 roles
    // (gemm8 reads the packed e4m3 weights) nor for the LayerNorm-folded QKV / c_fc (their fold
    // branch packs the row-major operand only)
    const bool wblk = h->w_blk != 0;
    for (int i = 0; i < h->cfg.layers; ++i) {
        LayerW& ly = h->layers[i];
        HIPCHK(alloc16(ly.wqkv, 3 * D * D));
        HIPCHK(alloc16(ly.wout, D * D));
        HIPCHK(alloc16(ly.wfc, 4 * D * D));
        HIPCHK(alloc16(ly.wproj, 4 * D * D));
        if (wblk && !h->q8_attn(i)) {
            if (!h->lnfold) HIPCHK(alloc16(ly.wqkv_b, 3 * D * D));
            HIPCHK(alloc16(ly.wout_b, D * D));
        }
        if (wblk && !h->q8_mlp(i)) {
            if (!h->lnfold) HIPCHK(alloc16(ly.wfc_b, 4 * D * D));
            HIPCHK(alloc16(ly.wproj_b, 4 * D * D));
        }
        ly.bqkv = h->master[L(i, "attn.in_proj_bias")];
        ly.bout = h->master[L(i, "attn.out_proj.bias")];
        ly.bfc = h->master[L(i, "mlp.c_fc.bias")];
        ly.bproj = h->master[L(i, "mlp.c_proj.bias")];
        ly.ln1g = h->master[L(i, "ln_1.weight")];
        ly.ln1b = h->master[L(i, "ln_1.bias")];
        ly.ln2g = h->master[L(i, "ln_2.weight")];
        ly.ln2b = h->master[L(i, "ln_2.bias")];
        maxw = std::max(maxw, 4 * D * D);
        if (h->lnfold) {
            if (!ly.s_qkv) HIPCHK(hipMalloc((void**)&ly.s_qkv, 3 * D * sizeof(float)));
            if (!ly.bf_qkv) HIPCHK(hipMalloc((void**)&ly.bf_qkv, 3 * D * sizeof(float)));
            if (!ly.s_fc) HIPCHK(hipMalloc((void**)&ly.s_fc, 4 * D * sizeof(float)));
            if (!ly.bf_fc) HIPCHK(hipMalloc((void**)&ly.bf_fc, 4 * D * sizeof(float)));
        }
    }
    if (h->lnfold && !h->scratch2) HIPCHK(hipMalloc((void**)&h->scratch2, 4 * D * D * sizeof(float)));
    if (h->scratch_elems < maxw) {
        if (h->scratch) hipFree(h->scratch);
        HIPCHK(hipMalloc(&h->scratch, maxw * sizeof(float)));
        h->scratch_elems = maxw;
    }
    hipStream_t s = nullptr;
    launch_patch_weight_relayout(s, h->master["visual.conv1.weight"], h->scratch, (int)D, h->cfg.patch_size);
    launch_pack_weight(s, h->dt, h->scratch, h->wpatch, (int)D, h->K3, h->Kp);
    launch_blk16_relayout(s, h->wpatch, h->wpatch_b, (int)D, h->Kp);
    for (int i = 0; i < h->cfg.layers; ++i) {
        LayerW& ly = h->layers[i];
        pack_linear(h, s, L(i, "attn.in_proj_weight"), ly.wqkv, nullptr);
        pack_linear(h, s, L(i, "attn.out_proj.weight"), ly.wout, nullptr);
        pack_linear(h, s, L(i, "mlp.c_fc.weight"), ly.wfc, nullptr);
        pack_linear(h, s, L(i, "mlp.c_proj.weight"), ly.wproj, nullptr);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    if (h->pool.empty()) {
        Workspace* w = nullptr;
        int rc = alloc_ws(h, &w);
        if (rc) return rc;
        h->pool.push_back(w);
    }
    h->loaded = true;
    return 0;
}

int clipvit_load_lora(clipvit_handle* h, const clipvit_lora* items, size_t n) {
    g_err.clear();
    if (!h || (!items && n)) FAIL(CLIPVIT_E_INVALID, "null argument");
    if (!h->loaded) FAIL(CLIPVIT_E_STATE, "weights not loaded");
    DeviceGuard dg(h->device);
    // map target -> packed destination
    std::unordered_map<std::string, void*> dst;
    for (int i = 0; i < h->cfg.layers; ++i) {
        dst[L(i, "attn.in_proj_weight")] = h->layers[i].wqkv;
        dst[L(i, "attn.out_proj.weight")] = h->layers[i].wout;
        dst[L(i, "mlp.c_fc.weight")] = h->layers[i].wfc;
        dst[L(i, "mlp.c_proj.weight")] = h->layers[i].wproj;
    }
    for (size_t k = 0; k < n; ++k) {
        const clipvit_lora& it = items[k];
        if (!it.target || !dst.count(it.target))
            FAIL(CLIPVIT_E_INVALID, std::string("unknown LoRA target ") + (it.target ? it.target : "(null)"));
        const auto& sh = h->shapes[it.target];
        if (sh[0] != it.out_features || sh[1] != it.in_features || it.rank <= 0 || !it.A || !it.B)
            FAIL(CLIPVIT_E_INVALID, std::string("LoRA shape mismatch for ") + it.target);
    }
    hipStream_t s = nullptr;
    // reset every Linear to its base weight, then merge each adapter (last call wins)
    for (auto& kv : dst) pack_linear(h, s, kv.first, kv.second, nullptr);
    std::unordered_map<std::string, std::vector<size_t>> groups;
    for (size_t k = 0; k < n; ++k) groups[items[k].target].push_back(k);
    for (auto& gkv : groups) {
        const auto& sh = h->shapes[gkv.first];
        const size_t cnt = (size_t)sh[0] * sh[1];
        HIPCHK(hipMemcpy(h->scratch, h->master[gkv.first], cnt * sizeof(float), hipMemcpyDeviceToDevice));
        for (size_t k : gkv.second) {
            const clipvit_lora& it = items[k];
            float *dA = nullptr, *dB = nullptr;
            HIPCHK(hipMalloc(&dA, (size_t)it.in_features * it.rank * sizeof(float)));
            HIPCHK(hipMalloc(&dB, (size_t)it.rank * it.out_features * sizeof(float)));
            HIPCHK(hipMemcpy(dA, it.A, (size_t)it.in_features * it.rank * sizeof(float), hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(dB, it.B, (size_t)it.rank * it.out_features * sizeof(float), hipMemcpyHostToDevice));
            launch_lora_merge(s, h->scratch, dA, dB, it.in_features, it.out_features, it.rank, it.scaling);
            HIPCHK(hipDeviceSynchronize());
            hipFree(dA);
            hipFree(dB);
        }
        pack_linear(h, s, gkv.first, dst[gkv.first], h->scratch);
        HIPCHK(hipDeviceSynchronize());
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    return 0;
}

int clipvit_set_text_features(clipvit_handle* h, const float* T, int C, int E, const int* seg_offsets,
                              int nseg) {
    g_err.clear();
    if (!h || !T || !seg_offsets) FAIL(CLIPVIT_E_INVALID, "null argument");
    if (E != h->E) FAIL(CLIPVIT_E_INVALID, "text feature width != embed_dim");
    if (C <= 0 || nseg <= 0) FAIL(CLIPVIT_E_INVALID, "empty text table");
    if (seg_offsets[0] != 0 || seg_offsets[nseg] != C)
        FAIL(CLIPVIT_E_INVALID, "seg_offsets must start at 0 and end at C");
    for (int i = 0; i < nseg; ++i)
        if (seg_offsets[i + 1] <= seg_offsets[i]) FAIL(CLIPVIT_E_INVALID, "empty or unordered segment");
    DeviceGuard dg(h->device);
    const int Cpad = (C + 63) / 64 * 64;
    std::vector<float> tt((size_t)E * Cpad, 0.f);
    for (int c = 0; c < C; ++c)
        for (int e = 0; e < E; ++e) tt[(size_t)e * Cpad + c] = T[(size_t)c * E + e];
    HIPCHK(hipDeviceSynchronize());  // no call may still read the old table
    if (h->Tt) hipFree(h->Tt);
    if (h->seg_dev) hipFree(h->seg_dev);
    h->Tt = nullptr;
    h->seg_dev = nullptr;
    HIPCHK(hipMalloc(&h->Tt, tt.size() * sizeof(float)));
    HIPCHK(hipMemcpy(h->Tt, tt.data(), tt.size() * sizeof(float), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&h->seg_dev, (nseg + 1) * sizeof(int)));
    HIPCHK(hipMemcpy(h->seg_dev, seg_offsets, (nseg + 1) * sizeof(int), hipMemcpyHostToDevice));
    h->seg_host.assign(seg_offsets, seg_offsets + nseg + 1);
    h->C = C;
    h->Cpad = Cpad;
    h->nseg = nseg;
    return 0;
}

int clipvit_text_shape(clipvit_handle* h, int* C, int* nseg) {
    if (!h) FAIL(CLIPVIT_E_INVALID, "null handle");
    if (C) *C = h->C;
    if (nseg) *nseg = h->nseg;
    return 0;
}

int clipvit_encode_image(clipvit_handle* h, void* stream, const void* pixels_dev, int dtype, int B,
                         float* emb_dev) {
    g_err.clear();
    int rc = check_call(h, pixels_dev, dtype, B);
    if (rc) return rc;
    if (!emb_dev) FAIL(CLIPVIT_E_INVALID, "null output");
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    Workspace* w = nullptr;
    if ((rc = acquire_ws(h, s, &w))) return rc;
    const size_t pxb = pixel_bytes(h, dtype);
    rc = run_lanes(h, s, B, w, [&](hipStream_t st, Lane* l, int off, int cnt) {
        return forward(h, st, (const char*)pixels_dev + off * pxb, dtype, cnt, l, emb_dev + (size_t)off * h->E,
                       nullptr);
    });
    release_ws(h, w);
    return rc;
}

int clipvit_classify(clipvit_handle* h, void* stream, const void* pixels_dev, int dtype, int B,
                     float* emb_dev, float* logits_dev, float* probs_dev, int32_t* top_idx,
                     float* top_prob) {
    g_err.clear();
    int rc = check_call(h, pixels_dev, dtype, B);
    if (rc) return rc;
    if (!h->Tt) FAIL(CLIPVIT_E_STATE, "text features not set");
    if (!logits_dev) FAIL(CLIPVIT_E_INVALID, "null logits buffer");
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    Workspace* w = nullptr;
    if ((rc = acquire_ws(h, s, &w))) return rc;
    const size_t pxb = pixel_bytes(h, dtype);
    const size_t C = h->C, E = h->E, T5 = (size_t)h->nseg * 5;
    rc = run_lanes(h, s, B, w, [&](hipStream_t st, Lane* l, int off, int cnt) {
        int r = forward(h, st, (const char*)pixels_dev + off * pxb, dtype, cnt, l, l->f, nullptr);
        if (r) return r;
        launch_logits(st, l->f, h->Tt, emb_dev ? emb_dev + off * E : nullptr, logits_dev + off * C, cnt, h->E,
                      h->C, h->Cpad, h->head_cols);
        if (probs_dev || top_idx || top_prob)
            launch_seg_softmax_topk(st, logits_dev + off * C, probs_dev ? probs_dev + off * C : nullptr,
                                    top_idx ? top_idx + off * T5 : nullptr,
                                    top_prob ? top_prob + off * T5 : nullptr, h->seg_dev, h->nseg, cnt,
                                    h->C);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            g_err = std::string("head launch failed: ") + hipGetErrorString(e);
            return CLIPVIT_E_HIP;
        }
        return 0;
    });
    release_ws(h, w);
    return rc;
}

int clipvit_gemm_log(clipvit_handle* h, int* out, int cap) {
    g_err.clear();
    if (!h || (!out && cap > 0) || cap < 0) FAIL(CLIPVIT_E_INVALID, "bad argument");
    std::lock_guard<std::mutex> lk(h->trace_mu);
    const int n = std::min(cap, (int)(h->trace_log.size() / 4));
    if (n) memcpy(out, h->trace_log.data(), (size_t)n * 4 * sizeof(int));
    h->trace_log.clear();
    return n;
}

int clipvit_profile_forward(clipvit_handle* h, void* stream, const void* pixels_dev, int dtype, int B,
                            int iters, float* out_ms) {
    g_err.clear();
    int rc = check_call(h, pixels_dev, dtype, B);
    if (rc) return rc;
    if (!out_ms || iters <= 0) FAIL(CLIPVIT_E_INVALID, "bad profile arguments");
    DeviceGuard dg(h->device);
    hipStream_t s = (hipStream_t)stream;
    Workspace* w = nullptr;
    if ((rc = acquire_ws(h, s, &w))) return rc;
    // One lane's forward, serialised on the caller's stream, at the per-lane batch the split
    // path launches (ceil(B/2) for B >= SPLIT_MIN): per-launch kernel times, no overlap.
    const int Bl = std::min(lane_batch(h, B), w->lane[0].cap);
    Lane* l = &w->lane[0];
    HIPCHK(hipStreamWaitEvent(s, l->done, 0));
    Prof p;
    const size_t nmarks = 8 + 8 * (size_t)h->cfg.layers;
    p.ev.resize(nmarks);
    p.fam.resize(nmarks);
    for (auto& e : p.ev) hipEventCreate(&e);
    double acc[F_COUNT] = {0};
    for (int it = 0; it < iters && !rc; ++it) {
        p.k = 0;
        rc = forward(h, s, pixels_dev, dtype, Bl, l, l->f, &p);
        if (rc) break;
        hipEventSynchronize(p.ev[p.k - 1]);
        for (size_t k = 1; k < p.k; ++k) {
            float ms = 0.f;
            hipEventElapsedTime(&ms, p.ev[k - 1], p.ev[k]);
            acc[p.fam[k]] += ms;
        }
    }
    // intervals per family in one forward (an event closes every interval), and the device
    // time between two back-to-back events with no work between them: the per-interval cost of
    // the marks themselves, which the family times above include
    int cnt[F_COUNT] = {0};
    for (size_t k = 1; k < p.k; ++k) ++cnt[p.fam[k]];
    float gap = 0.f;
    if (!rc) {  // events of its own (p.ev holds 8 + 8 L, which a 1-layer model makes < 17)
        constexpr int NG = 17;
        hipEvent_t g[NG];
        for (auto& e : g) hipEventCreate(&e);
        for (int k = 0; k < NG; ++k) hipEventRecord(g[k], s);
        hipEventSynchronize(g[NG - 1]);
        float ms = 0.f;
        hipEventElapsedTime(&ms, g[0], g[NG - 1]);
        gap = ms / (NG - 1);
        for (auto& e : g) hipEventDestroy(e);
    }
    hipEventRecord(l->done, s);
    for (auto& e : p.ev) hipEventDestroy(e);
    release_ws(h, w);
    for (int f = 0; f < F_COUNT; ++f) out_ms[f] = (float)(acc[f] / iters);
    out_ms[F_COUNT] = (float)Bl;
    for (int f = 0; f < F_COUNT; ++f) out_ms[F_COUNT + 1 + f] = (float)cnt[f];
    out_ms[2 * F_COUNT + 1] = gap;
    return rc;
}

int clipvit_destroy(clipvit_handle* h) {
    if (!h) return 0;
    DeviceGuard dg(h->device);
    hipDeviceSynchronize();
    for (auto& kv : h->master) hipFree(kv.second);
    hipFree(h->wpatch);
    hipFree(h->wpatch_b);
    for (auto& ly : h->layers) {
        hipFree(ly.wqkv);
        hipFree(ly.wout);
        hipFree(ly.wfc);
        hipFree(ly.wqkv_b);
        hipFree(ly.wfc_b);
        hipFree(ly.wout_b);
        hipFree(ly.wproj_b);
        hipFree(ly.wproj);
    }
    hipFree(h->scratch);
    hipFree(h->scratch2);
    for (auto& ly : h->layers) {
        hipFree(ly.s_qkv);
        hipFree(ly.bf_qkv);
        hipFree(ly.s_fc);
        hipFree(ly.bf_fc);
    }
    hipFree(h->Tt);
    hipFree(h->seg_dev);
    for (auto* w : h->pool) free_ws(w);
    delete h;
    return 0;
}

// ---- kernel-level test entry points ----
// compute units of the current device (the persistent GEMMs' grid)
static int current_ncu() {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
        return 0;
    return n;
}

int clipvit_gemm_test(void* stream, int dtype, const void* A_dev, const void* W_dev,
                      const float* bias_dev, float* C_dev, int M, int N, int K, int epi, int variant) {
    g_err.clear();
    if (!A_dev || !W_dev || !C_dev) FAIL(CLIPVIT_E_INVALID, "null argument");
    if (dtype != CLIPVIT_BF16 && dtype != CLIPVIT_F16) FAIL(CLIPVIT_E_INVALID, "dtype");
    if (K % 64 || N % 64 || M <= 0) FAIL(CLIPVIT_E_INVALID, "K and N must be multiples of 64");
    hipStream_t s = (hipStream_t)stream;
    void* Wp = nullptr;
    HIPCHK(hipMallocAsync(&Wp, (size_t)N * K * 2, s));
    launch_pack_weight(s, dtype, (const float*)W_dev, Wp, N, K, K);
    // + 10000: W in the blocked layout (GemmArgs.blk_w); + 20000: A too (GemmArgs.blk_a, a
    // blocked copy of A_dev with the rows padded to 16); + 30000: both
    const bool wblk = (variant / 10000) & 1, ablk = ((variant / 10000) >> 1) & 1;
    variant %= 10000;
    if (wblk && N % 16) FAIL(CLIPVIT_E_INVALID, "blocked W needs N % 16 == 0");
    void* Ab = nullptr;
    if (ablk) {
        const int mp = (M + 15) / 16 * 16;
        HIPCHK(hipMallocAsync(&Ab, (size_t)mp * K * 2, s));
        HIPCHK(hipMemsetAsync(Ab, 0, (size_t)mp * K * 2, s));
        void* Ap = nullptr;  // A with zero padding rows, then relaid out
        HIPCHK(hipMallocAsync(&Ap, (size_t)mp * K * 2, s));
        HIPCHK(hipMemsetAsync(Ap, 0, (size_t)mp * K * 2, s));
        HIPCHK(hipMemcpyAsync(Ap, A_dev, (size_t)M * K * 2, hipMemcpyDeviceToDevice, s));
        launch_blk16_relayout(s, Ap, Ab, mp, K);
        HIPCHK(hipFreeAsync(Ap, s));
    }
    if (wblk) {  // relayout in place through a copy
        void* Wr = nullptr;
        HIPCHK(hipMallocAsync(&Wr, (size_t)N * K * 2, s));
        HIPCHK(hipMemcpyAsync(Wr, Wp, (size_t)N * K * 2, hipMemcpyDeviceToDevice, s));
        launch_blk16_relayout(s, Wr, Wp, N, K);
        HIPCHK(hipFreeAsync(Wr, s));
    }
    GemmArgs a{};
    a.A = ablk ? Ab : A_dev; a.W = Wp; a.bias = bias_dev; a.C = C_dev;
    a.M = M; a.N = N; a.K = K; a.ldc = N;
    a.ncu = current_ncu();
    a.blk_w = wblk;
    a.blk_a = ablk;
    a.xcd_n = variant / 100;  // variant = 100 * xcd_partition + tile variant
    variant %= 100;
    int rc;
    // 16-bit-output-only variants (81 / 82 / 98 LDS-staged; 62, 72-77 persistent), or epi 10 / 11 = 16-bit STORE / GELU on
    // any variant: run, then widen to fp32
    const bool staged = variant == 81 || variant == 82 || variant == 98 || variant == 62 || variant == 72 ||
                        variant == 74 || variant == 75 || variant == 77 || variant == 79;
    if (epi >= 20) {  // split-K into epi - 20 slices: C_dev = [S][M][N] fp32 partials, no bias
        a.ksplit = epi - 20;
        a.bias = nullptr;
        rc = launch_gemm(s, dtype, EPI_F32, a, variant);
    } else if (staged || epi >= 10) {
        if (epi >= 10) epi -= 10;
        if (epi == 2) {
            hipFreeAsync(Wp, s);
            if (Ab) hipFreeAsync(Ab, s);
            FAIL(CLIPVIT_E_INVALID, "variant has no residual epilogue");
        }
        void* C16 = nullptr;
        HIPCHK(hipMallocAsync(&C16, (size_t)M * N * 2, s));
        a.C = C16;
        rc = launch_gemm(s, dtype, epi == 0 ? EPI_STORE : EPI_GELU, a, variant);
        if (!rc) launch_widen16(s, dtype, C16, C_dev, (size_t)M * N);
        HIPCHK(hipFreeAsync(C16, s));
    } else {
        const int e = epi == 0 ? EPI_F32 : epi == 1 ? EPI_F32GELU : EPI_RESID;
        rc = launch_gemm(s, dtype, e, a, variant);
    }
    HIPCHK(hipFreeAsync(Wp, s));
    if (Ab) HIPCHK(hipFreeAsync(Ab, s));
    if (rc) FAIL(CLIPVIT_E_INVALID, "unsupported gemm shape/variant");
    HIPCHK(hipGetLastError());
    return 0;
}

int clipvit_residual_x24_test(void* stream, const float* x_dev, void* planes_dev, float* back_dev, size_t n) {
    g_err.clear();
    if (!x_dev || !planes_dev || !back_dev || n == 0 || n % 4) FAIL(CLIPVIT_E_INVALID, "bad argument");
    launch_x24_roundtrip((hipStream_t)stream, x_dev, planes_dev, back_dev, n);
    HIPCHK(hipGetLastError());
    return 0;
}

int clipvit_quant_mx8_test(void* stream, int in_dtype, const void* src_dev, int rows, int K,
                           unsigned char* q_dev, unsigned char* sq_dev) {
    g_err.clear();
    if (!src_dev || !q_dev || !sq_dev || rows <= 0 || K <= 0 || K % 32)
        FAIL(CLIPVIT_E_INVALID, "bad argument");
    if (in_dtype < 0 || in_dtype > 2) FAIL(CLIPVIT_E_INVALID, "in_dtype");
    launch_quant_mx8((hipStream_t)stream, in_dtype, src_dev, q_dev, sq_dev, rows, K);
    HIPCHK(hipGetLastError());
    return 0;
}

int clipvit_gemm_mx8_test(void* stream, const unsigned char* A8_dev, const unsigned char* sA_dev,
                          const float* W_dev, const float* bias_dev, void* C_dev,
                          unsigned char* sC_dev, int M, int N, int K, int epi, int variant) {
    g_err.clear();
    if (!A8_dev || !sA_dev || !W_dev || !C_dev || M <= 0) FAIL(CLIPVIT_E_INVALID, "null argument");
    if (K % 128 || N % 128) FAIL(CLIPVIT_E_INVALID, "K and N must be multiples of 128");
    if ((epi == 3 || epi == 4) && !sC_dev) FAIL(CLIPVIT_E_INVALID, "sC required for MX-fp8 output");
    if (epi < 0 || epi > 5) FAIL(CLIPVIT_E_INVALID, "epi");
    hipStream_t s = (hipStream_t)stream;
    unsigned char* Wq = nullptr;
    HIPCHK(hipMallocAsync((void**)&Wq, (size_t)N * K + (size_t)N * K / 32, s));
    launch_pack_weight_mx8(s, W_dev, Wq, Wq + (size_t)N * K, N, K, K);
    GemmArgs a{};
    a.A = A8_dev; a.sA = sA_dev; a.W = Wq; a.sW = Wq + (size_t)N * K;
    a.bias = bias_dev; a.C = C_dev; a.sC = sC_dev;
    a.M = M; a.N = N; a.K = K; a.ldc = N;
    a.ncu = current_ncu();
    a.xcd_n = variant / 100;
    static const int emap[6] = {EPI_F32, EPI_F32GELU, EPI_RESID, EPI_Q8, EPI_GELU_Q8, EPI_STORE};
    const int rc = launch_gemm_mx8(s, CLIPVIT_BF16, emap[epi], a, variant % 100);
    HIPCHK(hipFreeAsync(Wq, s));
    if (rc) FAIL(CLIPVIT_E_INVALID, "unsupported MX-fp8 gemm shape/variant");
    HIPCHK(hipGetLastError());
    return 0;
}

int clipvit_gemm_bench(int dtype, int M, int N, int K, int epi, int variant, int iters,
                       float* avg_ms) {
    g_err.clear();
    if (!avg_ms || iters <= 0 || K % 64 || N % 64 || M <= 0) FAIL(CLIPVIT_E_INVALID, "bad argument");
    // dtype CLIPVIT_MXFP8: the MX-fp8 GEMM on random e4m3 operands (unit scales); epi 1
    // (QuickGELU) runs as the production EPI_GELU_Q8, 3 (patch) is not an MX-fp8 role
    const bool mx = dtype == CLIPVIT_MXFP8;
    if (mx && (K % 128 || epi == EPI_PATCH)) FAIL(CLIPVIT_E_INVALID, "unsupported MX-fp8 bench shape");
    void *A = nullptr, *W = nullptr, *Cb = nullptr;
    float* bias = nullptr;
    HIPCHK(hipMalloc(&A, (size_t)M * K * 2));
    HIPCHK(hipMalloc(&W, (size_t)N * K * 2));
    HIPCHK(hipMalloc(&Cb, (size_t)M * N * 4));
    HIPCHK(hipMalloc(&bias, (size_t)N * 4));
    if (mx) {
        launch_fill_random_mx8(nullptr, (unsigned char*)A, (unsigned char*)A + (size_t)M * K, (size_t)M * K, 1u);
        launch_fill_random_mx8(nullptr, (unsigned char*)W, (unsigned char*)W + (size_t)N * K, (size_t)N * K, 2u);
    } else {
        launch_fill_random16(nullptr, dtype, A, (size_t)M * K, 1u);
        launch_fill_random16(nullptr, dtype, W, (size_t)N * K, 2u);
    }
    HIPCHK(hipMemset(bias, 0, (size_t)N * 4));
    HIPCHK(hipMemset(Cb, 0, (size_t)M * N * 4));
    GemmArgs a{};
    a.A = A; a.W = W; a.bias = bias; a.C = Cb;
    a.M = M; a.N = N; a.K = K; a.ldc = N;
    a.patch_g2 = 49; a.patch_ntok = 50;
    // + 10000: blocked W, + 20000: blocked A, + 30000: both (random operands: the layout only
    // changes the access pattern)
    a.blk_w = (variant / 10000) & 1;
    a.blk_a = ((variant / 10000) >> 1) & 1;
    variant %= 10000;
    if (a.blk_w && N % 16) FAIL(CLIPVIT_E_INVALID, "blocked W needs N % 16 == 0");
    if (a.blk_a && M % 16) FAIL(CLIPVIT_E_INVALID, "blocked A needs M % 16 == 0");
    a.xcd_n = variant / 100;
    variant %= 100;
    a.ncu = current_ncu();
    int e = epi;  // raw Epi enum
    if (mx) {
        a.sA = (const unsigned char*)A + (size_t)M * K;
        a.sW = (const unsigned char*)W + (size_t)N * K;
        a.sC = (unsigned char*)Cb + (size_t)M * N;
        if (e == EPI_GELU) e = EPI_GELU_Q8;
    }
    auto launch = [&]() {
        return mx ? launch_gemm_mx8(nullptr, CLIPVIT_BF16, e, a, variant) : launch_gemm(nullptr, dtype, e, a, variant);
    };
    int rc = launch();
    hipEvent_t t0, t1;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    hipEventRecord(t0, nullptr);
    for (int i = 0; i < iters && !rc; ++i) rc = launch();
    hipEventRecord(t1, nullptr);
    hipEventSynchronize(t1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, t0, t1);
    hipEventDestroy(t0);
    hipEventDestroy(t1);
    *avg_ms = ms / iters;
    hipFree(A);
    hipFree(W);
    hipFree(Cb);
    hipFree(bias);
    if (rc) FAIL(CLIPVIT_E_INVALID, "unsupported variant/shape");
    HIPCHK(hipGetLastError());
    return 0;
}

int clipvit_attention_test(void* stream, int dtype, const void* qkv_dev, void* out_dev, int B, int N,
                           int H, int causal) {
    g_err.clear();
    if (!qkv_dev || !out_dev || B <= 0 || N <= 0 || H <= 0) FAIL(CLIPVIT_E_INVALID, "bad argument");
    // causal: bit 0 = causal mask; causal >> 4 = workgroups per CU of the persistent one-key-block
    // kernel (tuning attn_persist; 0 = one workgroup per unit)
    launch_attention((hipStream_t)stream, dtype, qkv_dev, out_dev, B, N, H, (causal & 1) != 0, causal >> 4, current_ncu());
    HIPCHK(hipGetLastError());
    return 0;
}

}  // extern "C"
