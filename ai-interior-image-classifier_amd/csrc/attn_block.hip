// One image's attention sub-block in one workgroup (ViT-B/32: N <= 64 tokens, D = 768, 12 heads):
//   O = MHA(qkv)                       (attention_v2_kernel<SINGLE>'s arithmetic per head)
//   y = fp16(O @ W_out^T + b_out)      (out_proj, the 16-bit branch output)
//   x = x + y  -> the 24-bit residual planes, in place
//   h = LayerNorm_2(x) -> c_fc's A operand in the 16-row blocked layout (blk16_off)
// Reference: ResidualAttentionBlock.forward's `x = x + attn(ln_1(x))` and the `ln_2(x)` that
// feeds the MLP [3p], reached from model.encode_image at main.py:204 / main.py:444 / main.py:503.
//
// Why one kernel: at N = 50 the three unfused kernels (attention, the out_proj
// GEMM, the add + LayerNorm) move the attention output O and the branch output y through memory
// twice each, and the attention kernel is latency-bound (one (image, head) per workgroup). Here
// a workgroup owns one image: O stays in LDS (64 x 768 fp16, 96 KB), out_proj streams W_out
// (1.2 MB, shared by every CU of an XCD, so L2-resident) through registers, and the LayerNorm
// has whole rows in the workgroup. One workgroup per image = 256 at bs 256 (one per CU).
//
// LDS: O [64 rows][1536 B], 16-B chunk c of row r at chunk c ^ (r & 15) (conflict-free
// ds_read_b128 of the out_proj A fragments); then two K/V stages of two heads each
// ([K 64 x 128 B | V 64 x 128 B] per head, attention_v2's swizzled image): 96 + 64 = 160 KB.
// Waves 0-3 run the even head of a pair, waves 4-7 the odd one; the next pair's K/V (LDS-DMA)
// and Q (registers) are in flight while a pair is computed.
// out_proj: wave w owns packed W rows [96 w, 96 w + 96) (6 fragments of 16) for all 64 token
// rows (4 fragments): 24 accumulators of 16x16, swapped operands as every GEMM here
// (acc = mfma(W, O)), W fragments loaded straight from the blocked packed copy (one 1 KB run per
// fragment and 32-deep k-step), one k-step ahead.
#include "common.h"

namespace clipvit {

typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));

template <typename T>
__global__ __launch_bounds__(512, 1) void attn_out_ln_kernel(const u16* __restrict__ qkv,
                                                             const unsigned char* __restrict__ wob,
                                                             const float* __restrict__ bout,
                                                             unsigned char* __restrict__ x24, size_t plane,
                                                             const float* __restrict__ g2,
                                                             const float* __restrict__ b2, u16* __restrict__ hout,
                                                             int N) {
    typedef typename T::vec8 vec8;
    constexpr int D = 768, H = 12, LD = 3 * D, OROW = 2 * D;  // O row pitch 1536 B
    constexpr int OB = 64 * OROW, KVST = 2 * 2 * 8192;        // 96 KB; one K/V stage = 32 KB
    __shared__ __attribute__((aligned(16))) unsigned char smem[OB + 2 * KVST];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, g = lane >> 4;
    const size_t base = (size_t)blockIdx.x * N;  // first token row of this image

    // ---------------- attention, two heads at a time ----------------
    const int grp = wave >> 2, wq = wave & 3;
    const int q = 16 * wq + j, qc = min(q, N - 1);
    const unsigned range = (unsigned)((size_t)(N - 1) * LD * 2 + (size_t)D * 2 + 128);
    auto issue = [&](int pair, int st) {  // K / V of head 2 pair + grp -> stage st (rows >= N: zeros)
        const int h = 2 * pair + grp;
        const i32x4_t rs = buf_rsrc(qkv + base * LD + D + h * 64, range);
        unsigned char* dst = smem + OB + st * KVST + grp * 16384;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int row = wq * 16 + r * 8 + (lane >> 3);
            const int c = (lane & 7) ^ (row & 7);
            const unsigned off = (unsigned)(row * LD * 2 + c * 16);
            blds16(rs, off, 0, dst + (wq * 16 + r * 8) * 128);
            blds16(rs, off + (unsigned)D * 2, 0, dst + 8192 + (wq * 16 + r * 8) * 128);
        }
    };
    auto loadq = [&](int pair, vec8 (&qf)[2]) {
        const u16* qrow = qkv + (base + qc) * LD + (2 * pair + grp) * 64;
        qf[0] = *(const vec8*)(qrow + 8 * g);
        qf[1] = *(const vec8*)(qrow + 32 + 8 * g);
    };
    const float scale = 0.125f;  // 1/sqrt(64)
    auto head = [&](int pair, const vec8 (&qf)[2]) {
        const int h = 2 * pair + grp;
        const unsigned char* Ks = smem + OB + (pair & 1) * KVST + grp * 16384;
        const unsigned char* Vs = Ks + 8192;
        f32x4 s[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int row = kt * 16 + j;
#pragma unroll
            for (int ds = 0; ds < 2; ++ds) {
                const int c = ((ds << 2) | g) ^ (row & 7);
                const vec8 kf = *(const vec8*)(Ks + row * 128 + (c << 4));
                s[kt] = T::mfma16(kf, qf[ds], s[kt]);
            }
        }
        float mloc = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = kt * 16 + 4 * g + r;
                const float v = key < N ? s[kt][r] * scale : -INFINITY;
                s[kt][r] = v;
                mloc = fmaxf(mloc, v);
            }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        float l = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = __expf(s[kt][r] - mloc);
                s[kt][r] = p;
                l += p;
            }
        f32x4 o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        // V^T fragments by transposed reads (attention_v2_kernel: inline asm, then lgkmcnt(0))
        const int tq = (lane & 15) >> 2, tp = lane & 3;
        const unsigned vbase = (unsigned)(size_t)(LDS_AS const unsigned char*)Vs;
#pragma unroll
        for (int stp = 0; stp < 2; ++stp) {
            u32x2_t vr[4][2];
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    const int k = 32 * stp + 16 * hf + 4 * g + tq;
                    const int cl = 2 * dt + (tp >> 1);
                    const unsigned addr = vbase + k * 128 + ((cl ^ (k & 7)) << 4) + 8 * (tp & 1);
                    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(vr[dt][hf]) : "v"(addr) : "memory");
                }
            vec8 pf;
            {
                unsigned w[4] = {pack2<T>(s[2 * stp][0], s[2 * stp][1]), pack2<T>(s[2 * stp][2], s[2 * stp][3]),
                                 pack2<T>(s[2 * stp + 1][0], s[2 * stp + 1][1]),
                                 pack2<T>(s[2 * stp + 1][2], s[2 * stp + 1][3])};
                pf = __builtin_bit_cast(vec8, *(uint4*)w);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const uint4 vv = make_uint4(vr[dt][0].x, vr[dt][0].y, vr[dt][1].x, vr[dt][1].y);
                o[dt] = T::mfma16(__builtin_bit_cast(vec8, vv), pf, o[dt]);
            }
        }
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        const float inv = 1.0f / l;
        // O[q][64 h + 16 dt + 4 g + r] (the bytes attention_v2 stores), into the swizzled O image
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const uint2 w = make_uint2(pack2<T>(o[dt][0] * inv, o[dt][1] * inv), pack2<T>(o[dt][2] * inv, o[dt][3] * inv));
            const int c = 8 * h + 2 * dt + (g >> 1);
            *(uint2*)(smem + q * OROW + ((c ^ (q & 15)) << 4) + (g & 1) * 8) = w;
        }
    };

    // ATTB_ABL (diagnostic builds only, outputs garbage): 1 = no attention phase, 2 = no out_proj
    // k-loop
#ifndef ATTB_ABL
#define ATTB_ABL 0
#endif
    vec8 qa[2], qb[2];
    if constexpr (ATTB_ABL != 1) {
    issue(0, 0);
    loadq(0, qa);
#pragma unroll
    for (int pair = 0; pair < H / 2; ++pair) {
        vec8 (&qc_)[2] = (pair & 1) ? qb : qa;
        vec8 (&qn_)[2] = (pair & 1) ? qa : qb;
        if (pair + 1 < H / 2) {
            issue(pair + 1, (pair + 1) & 1);
            loadq(pair + 1, qn_);
            vm_wait<6>();  // this pair's 4 pieces + 2 Q loads landed; the next pair's 6 may fly
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();  // every wave's pieces of this pair
        head(pair, qc_);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's stage reads and O writes
        __builtin_amdgcn_s_barrier();        // before the stage is refilled / O is read
    }
    }

    // ---------------- out_proj: y^T[n][t] = W_out[n] . O[t] ----------------
    const unsigned char* wl = wob + (size_t)(6 * wave) * 24576 + lane * 16;  // fragment fn: + fn * 24576
    f32x4 acc[6][4];
#pragma unroll
    for (int fn = 0; fn < 6; ++fn)
#pragma unroll
        for (int fm = 0; fm < 4; ++fm) acc[fn][fm] = f32x4{0.f, 0.f, 0.f, 0.f};
    // ATTB_ROT (A/B knob): workgroup b starts its k-steps at (b * ATTB_ROT) mod 24, so the CUs of
    // an XCD do not all read the same W_out lines at once (changes the summation order per image)
#ifndef ATTB_ROT
#define ATTB_ROT 0
#endif
    const int k0 = (int)((blockIdx.x * ATTB_ROT) % (D / 32));
    auto wk = [&](int kk) {
        const int k1 = kk + k0 >= D / 32 ? kk + k0 - D / 32 : kk + k0;
        return (k1 >> 1) * 2048 + (k1 & 1) * 1024;
    };
    vec8 wa[6], wb[6];
#pragma unroll
    for (int fn = 0; fn < 6; ++fn) wa[fn] = *(const vec8*)(wl + fn * 24576 + wk(0));
#pragma unroll
    for (int kk = 0; kk < (ATTB_ABL == 2 ? 0 : D / 32); ++kk) {
        vec8 (&wc)[6] = (kk & 1) ? wb : wa;
        vec8 (&wn)[6] = (kk & 1) ? wa : wb;
        if (kk + 1 < D / 32) {
            const int o1 = wk(kk + 1);
#pragma unroll
            for (int fn = 0; fn < 6; ++fn) wn[fn] = *(const vec8*)(wl + fn * 24576 + o1);
        }
        const int kr = kk + k0 >= D / 32 ? kk + k0 - D / 32 : kk + k0;
        vec8 af[4];
#pragma unroll
        for (int fm = 0; fm < 4; ++fm) {
            const int row = 16 * fm + j;
            const int c = (4 * kr + g) ^ j;  // (row & 15) == j
            af[fm] = *(const vec8*)(smem + row * OROW + (c << 4));
        }
#pragma unroll
        for (int fn = 0; fn < 6; ++fn)
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) acc[fn][fm] = T::mfma16(wc[fn], af[fm], acc[fn][fm]);
    }

    // ---------------- y = fp16(acc + b); x += y; h = LN_2(x) ----------------
    // Row phase, as add_layernorm_kernel: wave w takes token rows t = w, w + 8, ... (< N); a lane
    // holds columns 4 (lane + 64 i) .. + 3, i < 3, so the residual planes are read and written in
    // whole rows and the LayerNorm statistics are wave sums (add_layernorm_kernel's arithmetic).
    // The row loads are issued first; y goes through LDS ([64][768] fp16, the dead O image).
    constexpr int RPW = 8;  // row slots per wave (64 token rows / 8 waves)
    float4 xr[RPW][3];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int t = min(wave + 8 * r, N - 1);
#pragma unroll
        for (int i = 0; i < 3; ++i) xr[r][i] = x24_load(x24, plane, (base + t) * D + (lane + 64 * i) * 4);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();  // every wave is done reading O
    // lane (j, g) of fragment (fn, fm): token t = 16 fm + j, packed row p = 96 wave + 16 fn +
    // 4 g + r -> feature n = 64 (p >> 6) + 16 g + 4 ((p >> 4) & 3) + r (the packer's permutation)
    u16* Y = (u16*)smem;
#pragma unroll
    for (int fn = 0; fn < 6; ++fn) {
        const int pr = 96 * wave + 16 * fn;
        const int n = 64 * (pr >> 6) + 16 * g + 4 * ((pr >> 4) & 3);
        const float4 bb = *(const float4*)(bout + n);
#pragma unroll
        for (int fm = 0; fm < 4; ++fm) {
            const int t = 16 * fm + j;
            *(uint2*)(Y + t * D + n) = make_uint2(pack2<T>(acc[fn][fm][0] + bb.x, acc[fn][fm][1] + bb.y),
                                                  pack2<T>(acc[fn][fm][2] + bb.z, acc[fn][fm][3] + bb.w));
        }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int t = wave + 8 * r;
        if (t >= N) break;
        float4 v[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const uint2 w = *(const uint2*)(Y + t * D + (lane + 64 * i) * 4);
            v[i] = xr[r][i];
            v[i].x += T::to_f32((u16)(w.x & 0xffff));
            v[i].y += T::to_f32((u16)(w.x >> 16));
            v[i].z += T::to_f32((u16)(w.y & 0xffff));
            v[i].w += T::to_f32((u16)(w.y >> 16));
            x24_store(x24, plane, (base + t) * D + (lane + 64 * i) * 4, v[i]);
        }
        ln_row<3>(v, g2, b2, lane, (float)D);
#pragma unroll
        for (int i = 0; i < 3; ++i)
            gst<EW_AUX_ST>(hout, blk16_off((int)(base + t), (lane + 64 * i) * 4, D),
                           make_uint2(pack2<T>(v[i].x, v[i].y), pack2<T>(v[i].z, v[i].w)));
    }
}

// Returns -1 for shapes the kernel does not cover (the caller runs attention + out_proj GEMM +
// add + LayerNorm instead): D = 768 (12 heads), N <= 64, the blocked packed W_out copy present.
int launch_attn_out_ln(hipStream_t s, int dtype, const void* qkv, const void* wout_blk, const float* bout,
                       void* x24, size_t plane, const float* g2, const float* b2, void* h, int B, int N, int D) {
    if (D != 768 || N < 1 || N > 64 || !wout_blk || B < 1) return -1;
    const u16* q = (const u16*)qkv;
    const unsigned char* w = (const unsigned char*)wout_blk;
    unsigned char* x = (unsigned char*)x24;
    if (dtype == 2) attn_out_ln_kernel<F16><<<B, 512, 0, s>>>(q, w, bout, x, plane, g2, b2, (u16*)h, N);
    else attn_out_ln_kernel<BF16><<<B, 512, 0, s>>>(q, w, bout, x, plane, g2, b2, (u16*)h, N);
    return 0;
}

}  // namespace clipvit
