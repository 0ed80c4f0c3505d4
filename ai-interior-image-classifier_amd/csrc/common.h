// Shared device helpers and kernel-launcher declarations for libclipvit_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace clipvit {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

// Element tag types: storage is always 16-bit, T selects the MFMA operand format.
struct BF16 {
    typedef bf16x8 vec8;
    static __device__ __forceinline__ u16 from_f32(float f) {
        return __builtin_bit_cast(u16, (__bf16)f);
    }
    static __device__ __forceinline__ float to_f32(u16 v) {
        return __builtin_bit_cast(float, (unsigned)v << 16);
    }
    static __device__ __forceinline__ f32x4 mfma16(const vec8& a, const vec8& b, const f32x4& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};
struct F16 {
    typedef f16x8 vec8;
    static __device__ __forceinline__ u16 from_f32(float f) {
        return __builtin_bit_cast(u16, (_Float16)f);
    }
    static __device__ __forceinline__ float to_f32(u16 v) {
        return (float)__builtin_bit_cast(_Float16, v);
    }
    static __device__ __forceinline__ f32x4 mfma16(const vec8& a, const vec8& b, const f32x4& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
};

// Pack two fp32 into one dword of two 16-bit values (lo first): one v_cvt_pk_{f16,bf16}_f32 (RNE,
// the same rounding as two scalar conversions)
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
    if constexpr (__is_same(T, F16))
        return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){lo, hi}, f16x2_t));
    else
        return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}

// max over the four lanes l, l ^ 16, l ^ 32, l ^ 48 (the 16-lane rows of a wave) by the gfx950
// row-swap permutes (VALU; __shfl_xor is an LDS ds_bpermute round trip). Each swap exchanges
// rows between its two operands; max of the two results is max(v[l], v[l ^ 16]) (resp. ^ 32)
// in every lane, whichever operand received which half.
// CLIP's QuickGELU x sigmoid(1.702 x) = x / (1 + 2^(-1.702 log2(e) x)): one multiply by the folded
// constant, v_exp_f32, an add, v_rcp_f32 and the final multiply. Every GEMM epilogue and the
// split-K tail call this one function, so every tile's c_fc output is the same bits.
__device__ __forceinline__ float quick_gelu(float x) {
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-2.4554669595930157f * x));
}
// the same on two values (bit-identical): the multiplies and the add as v_pk_*_f32
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void quick_gelu2(float& a, float& b) {
    const f32x2 y = {a, b};
    const f32x2 z = y * (f32x2){-2.4554669595930157f, -2.4554669595930157f};
    const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)} + (f32x2){1.0f, 1.0f};
    const f32x2 o = y * (f32x2){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    a = o.x;
    b = o.y;
}

__device__ __forceinline__ float max_rows4(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// 16-byte async copy global -> LDS (global_load_lds_dwordx4). lds_wave_base must be the
// wave-uniform LDS destination; lane i lands at lds_wave_base + 16*i.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((const GLB_AS void*)gsrc, (LDS_AS void*)lds_wave_base, 16, 0,
                                     0);
}

// 16-byte async copy through a buffer resource -> LDS (buffer_load_dwordx4 ... offen lds):
// per-lane 32-bit byte offset voff (a VGPR that can stay constant across k-steps), wave-uniform
// soff (SGPR: the k offset), range-checked against the resource's byte count.
typedef int i32x4_t __attribute__((ext_vector_type(4)));
__device__ void raw_buffer_load_lds(i32x4_t rsrc, LDS_AS void* lds, int size, int voffset, int soffset, int offset,
                                    int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");
// raw (stride 0) buffer resource over [base, base + bytes); base and bytes wave-uniform
__device__ __forceinline__ i32x4_t buf_rsrc(const void* base, unsigned bytes) {
    const unsigned long long pa = (unsigned long long)base;
    i32x4_t r;
    r.x = (int)(unsigned)pa;
    r.y = (int)((unsigned)(pa >> 32) & 0xffffu);
    r.z = (int)bytes;
    r.w = 0x00020000;  // gfx9 raw buffer: DATA_FORMAT 32, no swizzle
    return r;
}
// AUX: the cache-policy bits of the load (gfx950: 1 sc0, 2 nt, 16 sc1)
template <int AUX = 0>
__device__ __forceinline__ void blds16(i32x4_t rsrc, unsigned voff, int soff, void* lds_wave_base) {
    raw_buffer_load_lds(rsrc, (LDS_AS void*)lds_wave_base, 16, (int)voff, soff, 0, AUX);
}
// 16-byte store through a buffer resource (buffer_store_dwordx4 ... offen): per-lane byte offset,
// range-checked (an offset past the resource's byte count writes nothing). aux 2 = non-temporal.
// A kernel whose counted vmcnt waits include its epilogue stores issues them this way, so the
// number of store instructions does not depend on how many rows are valid (a branch around an
// all-masked store would drop it from the count).
__device__ void raw_buffer_store_v4i32(i32x4_t data, i32x4_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v4i32");

// Cache policy of the GEMM epilogue stores (gfx950 bits: 1 sc0, 2 nt, 16 sc1). sc0 sc1 (17)
// writes the line through and drops it from the XCD's L2 (MI355X_MICROARCH.md, store flavours),
// so a tile's output does not evict the operand panels the XCD's other tiles are still reading.
// r06 same-box A/B on the 32-deep-k-step tile (QKV, c_fc): QKV 0.542 -> 0.523 ms, c_fc 0.676 ->
// 0.655 ms per forward, B/32 +1.2-1.5 % against plain stores; nt loads of A: -5 %
// (profiles/r06/store_policy_ab.txt).
#ifndef GEMM_ST_AUX
#define GEMM_ST_AUX 17
#endif
// 16-byte store at byte offset off of the buffer rs (wave-uniform base), with cache policy AUX
template <int AUX>
__device__ __forceinline__ void st16_pol(const i32x4_t& rs, size_t off, const uint4& v) {
    raw_buffer_store_v4i32(__builtin_bit_cast(i32x4_t, v), rs, (int)(unsigned)off, 0, AUX);
}
// 16-byte store at byte offset off (< 4 GB) of the wave-uniform base C: a plain global store for
// AUX 0, else a buffer store with those policy bits
template <int AUX>
__device__ __forceinline__ void cstore16(void* C, size_t off, const uint4& v) {
    if constexpr (AUX == 0) *(uint4*)((unsigned char*)C + off) = v;
    else st16_pol<AUX>(buf_rsrc(C, 0xFFFFFFFFu), off, v);
}
typedef int i32x2_t __attribute__((ext_vector_type(2)));
__device__ void raw_buffer_store_v2i32(i32x2_t data, i32x4_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v2i32");
__device__ void raw_buffer_store_i32(int data, i32x4_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.i32");
// 4-, 8- or 16-byte store at byte offset off (< 4 GB) of the wave-uniform base, cache policy AUX
// (0: a plain global store)
template <int AUX, typename V>
__device__ __forceinline__ void gst(void* base, size_t off, const V& v) {
    if constexpr (AUX == 0) {
        *(V*)((unsigned char*)base + off) = v;
    } else {
        const i32x4_t rs = buf_rsrc(base, 0xFFFFFFFFu);
        if constexpr (sizeof(V) == 16) raw_buffer_store_v4i32(__builtin_bit_cast(i32x4_t, v), rs, (int)(unsigned)off, 0, AUX);
        else if constexpr (sizeof(V) == 8) raw_buffer_store_v2i32(__builtin_bit_cast(i32x2_t, v), rs, (int)(unsigned)off, 0, AUX);
        else raw_buffer_store_i32(__builtin_bit_cast(int, v), rs, (int)(unsigned)off, 0, AUX);
    }
}
// store policy of the streaming kernels' outputs (the 24-bit residual planes, the LayerNorm
// kernels' blocked h, im2col): sc0 sc1. r06 same box, B/32 bs 256: LayerNorm family 0.366-0.372
// -> 0.351-0.359 ms per forward, +0.4-0.9 % (the attention output measured slower that way:
// attention.hip ATT_AUX_ST; profiles/r06/store_policy_ab.txt)
#ifndef EW_AUX_ST
#define EW_AUX_ST GEMM_ST_AUX
#endif
// store policy of the ping-pong (gemm_pp.hip: sc0 sc1, B/32 bs 128 +2.2 % same box, c_fc 0.48 ->
// 0.445 ms per forward) and MX-fp8 (mx8.hip, gemm_p32mx.h: plain; sc0 sc1 measured -6 % on config
// 5) tiles (profiles/r06/store_policy_ab.txt)
#ifndef PP_AUX_ST
#define PP_AUX_ST GEMM_ST_AUX
#endif
#ifndef MX_AUX_ST
#define MX_AUX_ST 0
#endif
#ifndef MX_AUX_ST16  // the MX tiles' 16-bit / fp32 outputs (MX_AUX_ST: their MX-fp8 outputs)
#define MX_AUX_ST16 0
#endif

// ---- MX-fp8: OCP e4m3 elements, one E8M0 (power-of-two) scale per 32 consecutive K ----
// Block rule (shared by every producer and by the tests' host reference): e = the smallest
// integer with amax * 2^-e <= 448 (e4m3's largest finite), clamped to [-127, 126]; scale byte
// = e + 127; element = RNE-e4m3(x * 2^-e). amax == 0 gives e = -127 and zero elements.
__device__ __forceinline__ int mx_exp(float amax) {
    if (!(amax > 0.f)) return -127;
    int ex;
    const float m = frexpf(amax * (1.0f / 448.0f), &ex);  // amax/448 = m 2^ex, m in [0.5, 1)
    int e = m == 0.5f ? ex - 1 : ex;
    return e < -127 ? -127 : (e > 126 ? 126 : e);
}
__device__ __forceinline__ float mx_inv(int e) { return __int_as_float((127 - e) << 23); }  // 2^-e
// four floats (already scaled) -> four e4m3 bytes, first value in the low byte
__device__ __forceinline__ unsigned pk4_e4m3(float a, float b, float c, float d) {
    unsigned r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
}

// s_waitcnt vmcnt(N) as inline asm (hand-counted waits of the glds pipelines)
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// GEMM epilogues.
enum Epi {
    EPI_STORE = 0,   // C (T)   = acc + bias
    EPI_GELU = 1,    // C (T)   = quickgelu(acc + bias)
    EPI_RESID = 2,   // C (f32) += acc + bias
    EPI_PATCH = 3,   // C (f32) [remapped token row] = acc          (conv1 has no bias)
    EPI_F32 = 4,     // C (f32) = acc + bias                         (tests)
    EPI_F32GELU = 5, // C (f32) = quickgelu(acc + bias)              (tests)
    EPI_GELU_Q8 = 7, // C (MX-fp8) = quickgelu(acc + bias), block scales to sC  (MX-fp8 GEMM)
    EPI_Q8 = 8,      // C (MX-fp8) = acc + bias, block scales to sC             (tests)
    // LayerNorm folded into the consumer GEMM: A = fp16(x) (the residual
    // stream, NOT normalised), W' = W diag(gamma); per row mu / rstd from the producer's
    // 128-column partial statistics st_in; bias = b' = b + W beta, lnf_s = s_n = sum_k W'_nk:
    EPI_LNF = 9,       // C (T) = rstd (acc - mu s_n) + b'_n                  = LN(x) W^T + b
    EPI_LNF_GELU = 10, // C (T) = quickgelu(rstd (acc - mu s_n) + b'_n)
    // residual producer: x (C, f32) += acc + bias; C2 (T) = x; st_out = per-row (mean, M2) of
    // x over every 128-column group (the consumer's LayerNorm statistics)
    EPI_RES_STATS = 11,
};

struct GemmArgs {
    const void* A;     // [M, K] activations (16-bit), row stride K
    const void* W;     // [N, K] packed weights (16-bit), row stride K
    const float* bias; // [N] or nullptr
    void* C;           // output, row stride ldc (elements)
    int M, N, K, ldc;
    int patch_g2, patch_ntok;  // EPI_PATCH row remap: m -> (m / g2) * ntok + 1 + m % g2
    int patch_R, patch_Rw;     // implicit patch GEMM: image side R, pixel row length Rw (A = [B, 3, R, Rw])
    int xcd_n;  // tile->XCD partition: 2 = 4 M-bands x 2 N-halves per XCD group (else 1-D)
    // MX-fp8 GEMM only: E8M0 block scales [rows][K/32] of A and W, [M][N/32] of a Q8 output
    const unsigned char* sA;
    const unsigned char* sW;
    unsigned char* sC;
    // LayerNorm fold (EPI_LNF*, EPI_RES_STATS): np = 128-column groups per row (D / 128)
    const float* lnf_s;
    const float2* st_in;
    float2* st_out;
    void* C2;
    int np;
    // split-K (EPI_F32 on the pipelined tiles only): grid.y = ksplit slices of K / ksplit each;
    // slice z writes its fp32 partial (no bias) to C + z * M * ldc. 0 / 1 = no split
    int ksplit;
    // compute units of the device the GEMM runs on: the persistent kernels' grid size
    // (0 = assume 256, MI355X)
    int ncu;
    // 16-row blocked layout (blk16_off) of the 16-bit A operand / C output: c_fc -> c_proj's u.
    // Pipelined (gemm_pipe_kernel) and persistent ping-pong (62 / 63) kernels only; the others
    // refuse it. Rows are padded to a multiple of 16 in the buffer.
    int blk_a, blk_c;
    // MX-fp8 u8 scales in the blocked form (with blk_a / blk_c): [K / 128][sc_rows] dwords, the
    // dword of (row, 128-deep k-tile) holding its four E8M0 bytes, so a k-tile's scales of
    // consecutive rows are one contiguous run (0 = row-major [rows][K / 32] bytes). sc_rows = the
    // padded row count of the whole matrix (a row-split launch passes its parent's)
    int sc_rows;
    // W in the 16-row blocked layout (blk16_off over its packed rows, launch_blk16_relayout): a
    // 64-deep k-tile of 16 weight rows is one contiguous 2 KB run. Pipelined tiles (8..98, not the
    // patch GEMM) and the persistent tiles (62 / 63 / 72 / 74) only.
    int blk_w;
    // EPI_RES_STATS: the residual x in 24-bit planes (x24_load / x24_store: C = the [M][ldc] u16
    // high plane, the byte plane at C + x24_plane); 0 = fp32 x at C
    size_t x24_plane;
};

// 16-row blocked layout of a 16-bit [rows, ncols] matrix (ncols % 64 == 0): 16 x 64 blocks of
// 2 KB, row-block-major; inside a block the eight 16-B feature chunks are stored chunk-major,
// 16 rows each. One 16-B column of 16 consecutive rows (what a quarter-wave of the MFMA
// accumulator layout holds) is then 256 contiguous bytes, and a 64-deep k-tile of a 16-row
// block is one contiguous 2 KB run (the consumer's LDS image verbatim). Byte offset of (m, f):
__host__ __device__ inline size_t blk16_off(int m, int f, int ncols) {
    return ((((size_t)(m >> 4) * (size_t)(ncols >> 6)) + (size_t)(f >> 6)) << 11) + (size_t)(((f & 63) >> 3) << 8) +
           (size_t)((m & 15) << 4) + (size_t)((f & 7) << 1);
}
// The same for a 1-byte (MX-fp8 e4m3) matrix, ncols % 128 == 0: 16 x 128 blocks of 2 KB, eight
// 16-byte feature chunks per block, chunk-major (the MX GEMM's 128-deep k-tile of a 16-row block
// is one contiguous 2 KB run). Byte offset of (m, f):
__host__ __device__ inline size_t blk8_off(int m, int f, int ncols) {
    return ((((size_t)(m >> 4) * (size_t)(ncols >> 7)) + (size_t)(f >> 7)) << 11) + (size_t)(((f & 127) >> 4) << 8) +
           (size_t)((m & 15) << 4) + (size_t)(f & 15);
}

// 24-bit residual rows (X24, the 16-bit forward): x as two planes, hi = the upper 16 bits of
// each fp32 value ([rows][D] u16 at base) and lo = the next 8 ([rows][D] bytes at base + plane),
// rounded to nearest at bit 8: a 16-bit significand (relative error <= 2^-16, against 2^-11 for
// the 16-bit GEMM operands), 3 bytes per element instead of 4. idx = row * D + column (4-aligned).
__device__ __forceinline__ float4 x24_load(const unsigned char* base, size_t plane, size_t idx) {
    const uint2 hi = *(const uint2*)(base + idx * 2);
    const unsigned lo = *(const unsigned*)(base + plane + idx);
    return make_float4(__uint_as_float((hi.x << 16) | ((lo & 0xffu) << 8)),
                       __uint_as_float((hi.x & 0xffff0000u) | (lo & 0xff00u)),
                       __uint_as_float((hi.y << 16) | ((lo >> 8) & 0xff00u)),
                       __uint_as_float((hi.y & 0xffff0000u) | ((lo >> 16) & 0xff00u)));
}
__device__ __forceinline__ void x24_store(unsigned char* base, size_t plane, size_t idx, float4 v) {
    const unsigned a = __float_as_uint(v.x) + 0x80u, b = __float_as_uint(v.y) + 0x80u;
    const unsigned c = __float_as_uint(v.z) + 0x80u, d = __float_as_uint(v.w) + 0x80u;
    gst<EW_AUX_ST>(base, idx * 2, make_uint2((a >> 16) | (b & 0xffff0000u), (c >> 16) | (d & 0xffff0000u)));
    gst<EW_AUX_ST>(base, plane + idx,
                   ((a >> 8) & 0xffu) | (b & 0xff00u) | ((c << 8) & 0xff0000u) | ((d << 16) & 0xff000000u));
}

// mean / rstd of a row from its np (mean, M2) partials over 128 columns each (Chan's combine,
// fixed order); eps 1e-5 as CLIP's LayerNorm
__device__ __forceinline__ void ln_fold_stats(const float2* __restrict__ st, int np, float& mu, float& rstd) {
    float s = 0.f;
    for (int p = 0; p < np; ++p) s += st[p].x;
    mu = s / (float)np;
    float m2 = 0.f;
    for (int p = 0; p < np; ++p) {
        const float d = st[p].x - mu;
        m2 += st[p].y + 128.f * d * d;
    }
    rstd = rsqrtf(m2 / (128.f * (float)np) + 1e-5f);
}

// Map a launch-order block id to its (m-tile, n-tile). Blocks b, b+8, ... are observed to
// share an XCD (speed only, never correctness). A 2-D partition gives every XCD group one cell
// of an XM x XN grid over (M-tiles, N-tiles): the group streams its M-band's A panels and keeps
// its share of W in its 4 MB L2; tiles inside a group run M-major. xn selects the grid:
// 2 = 4 x 2, 4 = 2 x 4, 8 = 1 x 8, 16 = 8 x 1 (XN must divide the N-tile count, else the 1-D
// bijective remap: each group takes a contiguous range of the row-major tile order).
__host__ __device__ inline int xcd_split_n(int nN, int xn) {
    const int XN = xn == 16 ? 1 : xn;
    return (xn == 2 || xn == 4 || xn == 8 || xn == 16) && nN % XN == 0 ? XN : 0;
}

__device__ __forceinline__ bool tile_of_block(int bid, int nM, int nN, int xn, int& mt, int& nt) {
    const int XN = xcd_split_n(nN, xn);
    if (XN) {
        const int XM = 8 / XN;
        const int x = bid & 7, j = bid >> 3;
        const int xm = x / XN, xh = x % XN;
        const int m_lo = (nM * xm) / XM, m_hi = (nM * (xm + 1)) / XM;
        const int nr = nN / XN, n_lo = xh * nr;
        if (j >= (m_hi - m_lo) * nr) return false;
        mt = m_lo + j / nr;
        nt = n_lo + j % nr;
        return true;
    }
    const int nwg = nM * nN;  // bijective 1-D remap: each group takes a contiguous range
    if (bid >= nwg) return false;
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    const int t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    // xn = 32 + G (G | nN): the contiguous ranges follow a column-group-major order (G groups of
    // nN / G N-tiles, M-rows inside a group), so an XCD group sweeps M with a 1/G share of W
    // (small enough for its L2) instead of all of W
    const int G = xn > 32 && nN % (xn - 32) == 0 ? xn - 32 : 1;
    const int cg = nN / G, gsz = nM * cg;
    const int g = t / gsz, rr = t - g * gsz;
    mt = rr / cg;
    nt = g * cg + rr % cg;
    return true;
}

// Grid size matching tile_of_block: 8 x (largest group) for a 2-D partition.
__host__ __device__ inline int grid_for(int nM, int nN, int xn) {
    const int XN = xcd_split_n(nN, xn);
    if (XN) {
        const int XM = 8 / XN;
        int mx = 0;
        for (int xm = 0; xm < XM; ++xm) {
            const int rows = ((nM * (xm + 1)) / XM) - ((nM * xm) / XM);
            mx = rows > mx ? rows : mx;
        }
        return 8 * mx * (nN / XN);
    }
    return nM * nN;
}

// Row LayerNorm helpers: one wave per row, D = 64 * 4 * V (V float4 per lane).
template <int V>
__device__ __forceinline__ void ln_row(float4 (&v)[V], const float* __restrict__ gm,
                                       const float* __restrict__ bt, int lane, float D) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    const float mean = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        v[i].x -= mean; v[i].y -= mean; v[i].z -= mean; v[i].w -= mean;
        q += (v[i].x * v[i].x + v[i].y * v[i].y) + (v[i].z * v[i].z + v[i].w * v[i].w);
    }
    const float rstd = rsqrtf(wave_sum(q) / D + 1e-5f);
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const int c = (lane + 64 * i) * 4;
        const float4 gg = *(const float4*)(gm + c), bb = *(const float4*)(bt + c);
        v[i].x = v[i].x * rstd * gg.x + bb.x;
        v[i].y = v[i].y * rstd * gg.y + bb.y;
        v[i].z = v[i].z * rstd * gg.z + bb.z;
        v[i].w = v[i].w * rstd * gg.w + bb.w;
    }
}

template <typename T, int V>
__device__ __forceinline__ void store_row16(u16* dst, const float4 (&v)[V], int lane) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const int c = (lane + 64 * i) * 4;
        *(uint2*)(dst + c) = make_uint2(pack2<T>(v[i].x, v[i].y), pack2<T>(v[i].z, v[i].w));
    }
}

// ---- launchers (defined in the .hip translation units) ----
// attention + out_proj + (x += y) + ln_2 of one block, one workgroup per image (attn_block.hip);
// -1 when the shape is not covered (D != 768, N > 64, no blocked W_out copy)
int launch_attn_out_ln(hipStream_t s, int dtype, const void* qkv, const void* wout_blk, const float* bout,
                       void* x24, size_t plane, const float* g2, const float* b2, void* h, int B, int N, int D);
void launch_add_layernorm_x24_store(hipStream_t s, int dtype, void* x24, const void* y, void* h, const float* g,
                                    const float* b, int rows, int D, int hblk);
// variant: 0 = auto by shape; tile variants listed in gemm.hip launch_t
int launch_gemm(hipStream_t s, int dtype, int epi, const GemmArgs& a, int variant);
// ping-pong 256x256 GEMM (gemm_pp.hip): variant 60 direct stores, 61 LDS-staged stores;
// EPI_STORE / EPI_GELU, N % 256 == 0, K % 128 == 0
int launch_gemm_pp(hipStream_t s, int dtype, int epi, const GemmArgs& a, int variant);
// implicit-GEMM patch embedding (no im2col): P = patch size (14, 16, 32), a.A = pixels
int launch_patch_gemm(hipStream_t s, int dtype, int P, const GemmArgs& a);
// pixels of any supported dtype -> 16-bit pixels of the compute type (same [B, 3, R, R] layout)
void launch_cast_pixels(hipStream_t s, int in_dtype, int out_dtype, const void* src, void* dst, size_t n);
// [B, 3, R, R] -> [B, 3, R, G * 16] 16-bit with every P-pixel patch row padded to 16 (zeros)
void launch_cast_pixels_padded(hipStream_t s, int in_dtype, int out_dtype, const void* src, void* dst, int B,
                               int R, int P);
// pixels [B, 3, R, R] -> the explicit patch GEMM's A: [roundup16(B G^2), Kp] 16-bit, 16-row blocked
// (blk16_off), k in the implicit patch GEMM's order; -1 on an unsupported P / Kp
int launch_im2col_blk(hipStream_t s, int in_dtype, int out_dtype, const void* src, void* dst, int B, int R, int P,
                      int Kp);
// conv1.weight [D, 3, P, P] fp32 -> [D, 3 * P * roundup8(P)] in the implicit patch GEMM's k order
void launch_patch_weight_relayout(hipStream_t s, const float* w, float* out, int D, int P);

// MX-fp8 path (mx8.hip). out16: 16-bit output type of EPI_STORE (1 bf16, 2 fp16).
int launch_gemm_mx8(hipStream_t s, int out16, int epi, const GemmArgs& a, int variant);
void launch_quant_mx8(hipStream_t s, int in_dtype, const void* src, unsigned char* q,
                      unsigned char* sq, int rows, int K);
void launch_fill_random_mx8(hipStream_t s, unsigned char* q, unsigned char* sq, size_t n, unsigned seed);
void launch_pack_weight_mx8(hipStream_t s, const float* src, unsigned char* q, unsigned char* sq,
                            int N, int K, int Kp);
// x16 (here and below): the fp16 residual stream of the MX-fp8 forward replaces fp32 x (nullptr: x)
void launch_add_layernorm(hipStream_t s, int dtype, float* x, const void* y, void* h, const float* g,
                          const float* b, int rows, int D, void* x16 = nullptr);
// x' = x + y (+ y2); h = LayerNorm(x'). y2 == nullptr: x' is NOT stored (deferred: the next
// call adds both branch outputs in the same order); y2 != nullptr: x' is stored.
// split-K reduction of the class-token tail (cls_tail): t = P[0] + ... + P[S-1] (fixed order),
// x += t + bias; with h != nullptr also h = LayerNorm(x) (16-bit)
void launch_splitk_resid_ln(hipStream_t s, int dtype, float* x, const float* P, int S, const float* bias,
                            void* h, const float* g, const float* b, int rows, int D);
// u = quickgelu(P[0] + ... + P[S-1] + bias) (16-bit), [rows, n]
void launch_splitk_gelu(hipStream_t s, int dtype, const float* P, int S, const float* bias, void* u, int rows,
                        int n);
// x24 = true: x16 is instead the 24-bit residual stream of the 16-bit forward (norm.hip x24_load);
// hblk (with x24): h in the 16-row blocked layout (blk16_off), rows padded to 16; 1 = direct
// stores, 2 = through an LDS transpose (norm.hip add_layernorm_kernel HBLK)
void launch_add_layernorm_deferred(hipStream_t s, int dtype, float* x, const void* y, const void* y2,
                                   void* h, const float* g, const float* b, int rows, int D, void* x16 = nullptr,
                                   bool x24 = false, int hblk = 0);
void launch_x24_roundtrip(hipStream_t s, const float* x, void* planes, float* back, size_t n);
void launch_gather_cls(hipStream_t s, const float* x, const void* h, float* xc, void* hc, int B, int N, int D,
                       const void* x16 = nullptr, bool x24 = false);
void launch_layernorm_q8(hipStream_t s, const float* x, unsigned char* q, unsigned char* sq,
                         const float* g, const float* b, int rows, int D);
// x (+)= y (+ y2), LayerNorm -> MX-fp8 q + scales sq (bf16 branch outputs of the MX-fp8 forward)
void launch_add_layernorm_q8(hipStream_t s, float* x, const void* y, const void* y2, unsigned char* q,
                             unsigned char* sq, const float* g, const float* b, int rows, int D, bool defer,
                             void* x16 = nullptr);
// x16 given: x holds the patch GEMM's fp32 rows (read only), the residual goes to x16 (fp16)
void launch_embed_ln_q8(hipStream_t s, float* x, unsigned char* q, unsigned char* sq,
                        const float* cls, const float* pos, const float* g_pre,
                        const float* b_pre, const float* g1, const float* b1, int B, int N, int D,
                        void* x16 = nullptr);

void launch_widen16(hipStream_t s, int dtype, const void* src, float* dst, size_t n);
// LayerNorm fold of a Linear (W [N, K] fp32, possibly LoRA-merged): Wg = W diag(gamma) (fp32,
// packed afterwards), s_n = sum_k fp16-or-bf16(Wg_nk), bo_n = b_n + sum_k W_nk beta_k
void launch_lnfold_prep(hipStream_t s, int dtype, const float* W, const float* gamma, const float* beta,
                        const float* b, float* Wg, float* s_out, float* b_out, int N, int K);
// embedding for the folded path: x = ln_pre(cls / patch + pos); x16 = x (16-bit); st = 128-col
// partial (mean, M2) of x; x24 (not null): x stored in the 24-bit planes there
void launch_embed_stats(hipStream_t s, int dtype, float* x, void* x16, float2* st, const float* cls,
                        const float* pos, const float* g_pre, const float* b_pre, int B, int N, int D,
                        void* x24 = nullptr);


// persist > 0 (N <= 64, non-causal): the persistent attention_p_kernel on persist workgroups per CU
// (ncu CUs; 0 = 256), else one workgroup per (image, head, 64-query block)
int launch_attention_q8(hipStream_t s, int dtype, const void* qkv, unsigned char* q8, unsigned char* q8s,
                        int B, int N, int H, int persist = 0, int ncu = 0);
void launch_attention(hipStream_t s, int dtype, const void* qkv, void* out, int B, int N, int H,
                      bool causal = false, int persist = 0, int ncu = 0);

void launch_embed_ln(hipStream_t s, int dtype, float* x, void* h, const float* cls,
                     const float* pos, const float* g_pre, const float* b_pre, const float* g1,
                     const float* b1, int B, int N, int D, void* x16 = nullptr, bool x24 = false);
void launch_layernorm(hipStream_t s, int dtype, const float* x, void* h, const float* g,
                      const float* b, int rows, int D);
void launch_pack_weight(hipStream_t s, int dtype, const float* src, void* dst, int N, int K,
                        int Kp);
void launch_blk16_relayout(hipStream_t s, const void* src, void* dst, int rows, int cols);
void launch_fill_random16(hipStream_t s, int dtype, void* p, size_t n, unsigned seed);
void launch_lora_merge(hipStream_t s, float* W, const float* A, const float* Bm, int in_f,
                       int out_f, int rank, float scaling);
void launch_cls_ln_proj(hipStream_t s, const float* x, const float* g, const float* b,
                        const float* proj, float* f, int B, int N, int D, int E, int tc = 64);
void launch_logits(hipStream_t s, const float* f, const float* Tt, float* emb_norm, float* logits,
                   int B, int E, int C, int Cpad, int tc = 64);
void launch_seg_softmax_topk(hipStream_t s, const float* logits, float* probs, int* top_idx,
                             float* top_prob, const int* seg_off, int nseg, int B, int C);

}  // namespace clipvit
