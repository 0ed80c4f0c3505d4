// Fused multi-head self-attention of the CLIP ViT vision tower (no mask):
//   O = softmax(Q K^T / sqrt(64)) V     per (image, head), head_dim 64
// Reference semantics: nn.MultiheadAttention inside OpenAI-CLIP ResidualAttentionBlock [3p]
// (packed in_proj, scale 1/sqrt(d_h), need_weights=False), reached from
// model.encode_image at main.py:204 / main.py:444 / main.py:503.
//
// Layout: qkv [B*N, 3*D] (16-bit, output of the QKV GEMM; q | k | v, head h at cols h*64),
//         out [B*N, D]   (16-bit, head h at cols h*64) -> input of the out_proj GEMM.
//
// One workgroup = 4 waves = 64 query rows of one (image, head) (attention_v2_kernel; each wave
// owns 16 queries) or 128 query rows (attention_v3_kernel, N > 128: 32 queries per wave).
// Keys/values are streamed in blocks of 64 through LDS with an online (flash-style) softmax,
// so any token count works: N = 50 (B/32, one key block), 77 (text, causal), 197 (B/16),
// 577 (L/14@336).
//   S^T[key][q] = mfma(K rows, Q rows)  -> lane (q = lane&15, g = lane>>4) holds 16 keys of
//                                           its own query: the row max/sum are 15 local ops +
//                                           two xor-shuffles (lanes q, q+16, q+32, q+48);
//   O^T[d][q]  += mfma(V^T, P^T)         -> P^T is consumed straight from the S registers
//                                           (permuted k order, matched on the V side), no LDS
//                                           round trip for P.
// K and V in LDS: 128-B rows, 16-B chunk swizzle c ^ (row & 7) (conflict-free ds_read_b128);
// V is read transposed by ds_read_b64_tr_b16.
#include "common.h"

namespace clipvit {

// ---------------------------------------------------------------------------------------
// attention_v2_kernel (the vision tower at N <= 128, and the causal text tower): K and V blocks
// reach LDS by buffer loads straight into LDS (async, no VGPR staging) into a 2-stage ring, so
// block kb+1 streams in while block kb is computed. V is stored row-major exactly like K (16-B
// chunk c ^ (key & 7)) and read TRANSPOSED by ds_read_b64_tr_b16: lane group g, lane 4q + p
// supplies key r0 + q, columns 4p .. 4p + 3; lane i receives column d = 16 dt + i of the 4
// keys — the A operand of O^T += V^T P^T with the k order of P (k-slot (g, e) <-> key
// 32 st + 16 (e >> 2) + 4 g + (e & 3)). No scalar LDS transposes, no __syncthreads (raw
// s_barrier + counted vmcnt keep the next block's loads in flight). Key rows past the sequence
// read as zeros (outside the rebased buffer range) and are masked to -inf in S.
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// QW waves per workgroup = 16 QW queries; every wave loads 64 / QW key rows of K and of V
// per block (long sequences run attention_v3_kernel instead, which halves the LDS reads).
// SINGLE (N <= 64, the B/32 shape): one key block, one LDS stage, no loop state — fewer live
// registers, so more workgroups per CU hide the load latency.
// CAUSAL (text tower): key j masked for query i < j; key blocks past the workgroup's last query
// are neither loaded nor computed.
// Q8 (MX-fp8 forward): the output goes straight to the out_proj operand format instead of 16-bit
// `out`: each value rounded to T first, then quantized by the launch_quant_mx8 rule, so the bytes
// equal attention + quant_mx8 exactly. MX block b of a head = features 32 b .. 32 b + 31 = the
// lane's dt 2b, 2b+1 values across the 4 lanes of its query (g = 0..3).
// store policy of the attention output (common.h gst; 0 = plain stores; sc0 sc1 measured
// slower: attention family 0.20 -> 0.22 ms per forward, profiles/r06/store_policy_ab.txt)
#ifndef ATT_AUX_ST
#define ATT_AUX_ST 0
#endif

template <typename T, int QW = 4, bool SINGLE = false, bool CAUSAL = false, bool Q8 = false>
__global__ __launch_bounds__(64 * QW, SINGLE ? 6 : 2) void attention_v2_kernel(const u16* __restrict__ qkv,
                                                                                u16* __restrict__ out, int N, int H,
                                                                                unsigned char* __restrict__ q8 = nullptr,
                                                                                unsigned char* __restrict__ q8s = nullptr) {
    typedef typename T::vec8 vec8;
    constexpr int STAGE = 2 * 64 * 128;  // K [64][128 B] | V [64][128 B]
    __shared__ __attribute__((aligned(16))) unsigned char smem[(SINGLE ? 1 : 2) * STAGE];

    const int D = H * 64;
    const int ld = 3 * D;
    const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, g = lane >> 4;
    const size_t base = (size_t)b * N;

    const int q = qb * (16 * QW) + wave * 16 + j;
    const int qc = min(q, N - 1);
    const u16* qrow = qkv + (base + qc) * ld + h * 64;
    vec8 qf[2];
    qf[0] = *(const vec8*)(qrow + 8 * g);
    qf[1] = *(const vec8*)(qrow + 32 + 8 * g);

    // glds assignment: wave w fills key rows [RW w, RW w + RW) of K and of V (1 KB pieces)
    constexpr int RW = 64 / QW, LPB = 2 * (RW / 8);  // rows per wave, glds per thread per block
    // K/V staging by buffer loads over this image's rows: per-lane offsets constant over the key
    // blocks. The resource is rebased at every key block (base += block offset, range -= block
    // offset: scalar arithmetic), because the hardware range check covers the per-lane offset
    // only, not an SGPR offset. Key rows >= N then lie past the range in every block and read
    // as zeros (their scores are masked, and P = 0 there); nothing past this image's last key row
    // is ever fetched (tests/test_gpu_kernels.py::test_attention_tail_rows_never_read).
    const unsigned char* src = (const unsigned char*)(qkv + base * ld + D + h * 64);
    const unsigned range = (unsigned)((size_t)(N - 1) * ld * 2 + (size_t)D * 2 + 128);
    auto issue = [&](int kb, int st) {
        unsigned char* dst = smem + st * STAGE;
        const unsigned kofs = (unsigned)(kb * 64 * ld * 2);
        const i32x4_t rs = buf_rsrc(src + kofs, range - kofs);
#pragma unroll
        for (int r = 0; r < RW / 8; ++r) {
            const int row = wave * RW + r * 8 + (lane >> 3);
            const int c = (lane & 7) ^ (row & 7);
            const unsigned off = (unsigned)(row * ld * 2 + c * 16);
            blds16(rs, off, 0, dst + (wave * RW + r * 8) * 128);
            blds16(rs, off + (unsigned)D * 2, 0, dst + 8192 + (wave * RW + r * 8) * 128);
        }
    };

    f32x4 o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;
    const float scale = 0.125f;  // 1/sqrt(64)
    int nkb = SINGLE ? 1 : (N + 63) >> 6;
    if constexpr (CAUSAL) nkb = min(nkb, (min(N - 1, qb * (16 * QW) + 16 * QW - 1) >> 6) + 1);

    issue(0, 0);
    if (!SINGLE && nkb > 1) issue(1, 1);
    for (int kb = 0; kb < nkb; ++kb) {
        const int st = kb & 1;
        if (kb + 1 < nkb) vm_wait<LPB>();  // block kb landed (this wave's part); kb+1 may fly
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();      // ... and every wave's part
        const unsigned char* Ks = smem + st * STAGE;
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
                const int key = kb * 64 + kt * 16 + 4 * g + r;
                const float v = key < N && (!CAUSAL || key <= q) ? s[kt][r] * scale : -INFINITY;
                s[kt][r] = v;
                mloc = fmaxf(mloc, v);
            }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float m_new = fmaxf(m_run, mloc);
        const float alpha = __expf(m_run - m_new);
        m_run = m_new;
        float lsum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = __expf(s[kt][r] - m_new);
                s[kt][r] = p;
                lsum += p;
            }
        l_run = l_run * alpha + lsum;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] *= alpha;

        // V^T fragments by transposed reads (inline asm: a builtin tr-read makes hipcc drain
        // vmcnt(0) before it, i.e. wait for the NEXT block's glds), then lgkmcnt(0) +
        // sched_barrier (hipcc would otherwise hoist the MFMAs past the wait)
        const int tq = (lane & 15) >> 2, tp = lane & 3;  // lane 4q + p of its 16-lane group
        const unsigned vbase = (unsigned)(size_t)(LDS_AS const unsigned char*)Vs;
#pragma unroll
        for (int stp = 0; stp < 2; ++stp) {  // one 32-key step at a time: 16 live V registers
            u32x2 vr[4][2];
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    const int k = 32 * stp + 16 * hf + 4 * g + tq;  // this lane's key row
                    const int cl = 2 * dt + (tp >> 1);               // logical chunk of d = 16 dt + 4 p
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
        if (!SINGLE && kb + 2 < nkb) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of the stage done
            __builtin_amdgcn_s_barrier();        // ... every wave's
            issue(kb + 2, st);
        }
    }

    l_run += __shfl_xor(l_run, 16, 64);
    l_run += __shfl_xor(l_run, 32, 64);
    if constexpr (Q8) {
        const float inv = 1.0f / l_run;
        float v[4][4], am[2] = {0.f, 0.f};
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
                const unsigned w = pack2<T>(o[dt][r] * inv, o[dt][r + 1] * inv);
                v[dt][r] = T::to_f32((u16)(w & 0xffff));
                v[dt][r + 1] = T::to_f32((u16)(w >> 16));
                am[dt >> 1] = fmaxf(am[dt >> 1], fmaxf(fabsf(v[dt][r]), fabsf(v[dt][r + 1])));
            }
#pragma unroll
        for (int bk = 0; bk < 2; ++bk) {
            am[bk] = fmaxf(am[bk], __shfl_xor(am[bk], 16, 64));
            am[bk] = fmaxf(am[bk], __shfl_xor(am[bk], 32, 64));
        }
        if (q < N) {
            const int e0 = mx_exp(am[0]), e1 = mx_exp(am[1]);
            const float i0 = mx_inv(e0), i1 = mx_inv(e1);
            unsigned char* qrow8 = q8 + (base + q) * D + h * 64;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const float iv = dt < 2 ? i0 : i1;
                *(unsigned*)(qrow8 + dt * 16 + 4 * g) =
                    pk4_e4m3(v[dt][0] * iv, v[dt][1] * iv, v[dt][2] * iv, v[dt][3] * iv);
            }
            if (g < 2) q8s[(base + q) * (D / 32) + h * 2 + g] = (unsigned char)((g == 0 ? e0 : e1) + 127);
        }
    } else if (q < N) {
        const float inv = 1.0f / l_run;
        const size_t orow = ((base + q) * D + h * 64) * 2;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            uint2 w;
            w.x = pack2<T>(o[dt][0] * inv, o[dt][1] * inv);
            w.y = pack2<T>(o[dt][2] * inv, o[dt][3] * inv);
            gst<ATT_AUX_ST>(out, orow + (dt * 16 + 4 * g) * 2, w);
        }
    }
}

// ---------------------------------------------------------------------------------------
// attention_p_kernel: the one-key-block attention (N <= 64, the ViT-B/32 shape) as a persistent
// loop. attention_v2<SINGLE> runs one (image, head) unit per workgroup: its K/V DMA, Q loads,
// 16 MFMAs and stores form one dependent chain of ~3 memory latencies per 25 KB moved, and at
// 8 workgroups per CU the chip is latency-bound (r06 profile: 4.3 TB/s of fabric traffic, wait
// share 0.36). Here a workgroup walks units u = blockIdx.x + i * gridDim.x with a 2-stage K/V
// ring: unit i + 1's K/V DMA and Q loads are issued before unit i is computed, so the loads of
// one unit overlap the arithmetic and stores of the previous one. Per unit the arithmetic is
// attention_v2<SINGLE>'s, instruction for instruction (the same bits).
template <typename T, bool Q8 = false>
__global__ __launch_bounds__(256, 2) void attention_p_kernel(const u16* __restrict__ qkv, u16* __restrict__ out, int B,
                                                            int N, int H, unsigned char* __restrict__ q8 = nullptr,
                                                            unsigned char* __restrict__ q8s = nullptr) {
    typedef typename T::vec8 vec8;
    constexpr int QW = 4, STAGE = 2 * 64 * 128;  // K [64][128 B] | V [64][128 B]
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];
    const int D = H * 64, ld = 3 * D;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, g = lane >> 4;
    const int q = wave * 16 + j, qc = min(q, N - 1);
    const int units = B * H, G = gridDim.x;
    constexpr int RW = 64 / QW, LPB = 2 * (RW / 8);  // K/V rows per wave; LDS-DMA pieces per wave and unit
    const unsigned range = (unsigned)((size_t)(N - 1) * ld * 2 + (size_t)D * 2 + 128);

    auto issue = [&](int u, int st) {  // unit u's K/V -> stage st (rows >= N read as zeros)
        const int b = u / H, h = u - b * H;
        const unsigned char* src = (const unsigned char*)(qkv + (size_t)b * N * ld + D + h * 64);
        const i32x4_t rs = buf_rsrc(src, range);
        unsigned char* dst = smem + st * STAGE;
#pragma unroll
        for (int r = 0; r < RW / 8; ++r) {
            const int row = wave * RW + r * 8 + (lane >> 3);
            const int c = (lane & 7) ^ (row & 7);
            const unsigned off = (unsigned)(row * ld * 2 + c * 16);
            blds16(rs, off, 0, dst + (wave * RW + r * 8) * 128);
            blds16(rs, off + (unsigned)D * 2, 0, dst + 8192 + (wave * RW + r * 8) * 128);
        }
    };
    // Q rows by inline-asm loads: invisible to hipcc's waitcnt pass, which would otherwise wait
    // for the NEXT unit's loads (vmcnt(0)) before the current unit's first MFMA; they are covered
    // by the counted wait below instead, and the two register sets alternate (no copies)
    auto load_q = [&](int u, vec8 (&qd)[2]) {
        const int b = u / H, h = u - b * H;
        const u16* qrow = qkv + ((size_t)b * N + qc) * ld + h * 64 + 8 * g;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qd[0]) : "v"(qrow) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off offset:64" : "=v"(qd[1]) : "v"(qrow) : "memory");
    };

    int u = blockIdx.x;
    if (u >= units) return;
    vec8 qa[2], qb[2];
    issue(u, 0);
    load_q(u, qa);
    const float scale = 0.125f;  // 1/sqrt(64)
    // one unit: K/V in stage st, Q in qf; prefetches the next unit's K/V / Q into stage st ^ 1 /
    // qn. Returns false after the workgroup's last unit.
    auto unit = [&](int st, vec8 (&qf)[2], vec8 (&qn)[2]) -> bool {
        const int un = u + G;
        const bool more = un < units;
        // the other stage was last read by the previous unit: every wave is past it (barrier at
        // the end of that unit)
        if (more) {
            issue(un, st ^ 1);
            load_q(un, qn);
            vm_wait<LPB + 2>();  // this unit's pieces and Q landed (the next unit's are the youngest LPB + 2)
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();  // ... every wave's
        const unsigned char* Ks = smem + st * STAGE;
        const unsigned char* Vs = Ks + 8192;

        f32x4 o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        float m_run = -INFINITY, l_run = 0.f;
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
        const float m_new = fmaxf(m_run, mloc);
        const float alpha = __expf(m_run - m_new);
        m_run = m_new;
        float lsum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = __expf(s[kt][r] - m_new);
                s[kt][r] = p;
                lsum += p;
            }
        l_run = l_run * alpha + lsum;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] *= alpha;
        const int tq = (lane & 15) >> 2, tp = lane & 3;
        const unsigned vbase = (unsigned)(size_t)(LDS_AS const unsigned char*)Vs;
#pragma unroll
        for (int stp = 0; stp < 2; ++stp) {
            u32x2 vr[4][2];
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
        l_run += __shfl_xor(l_run, 16, 64);
        l_run += __shfl_xor(l_run, 32, 64);
        const int b = u / H, h = u - b * H;
        const size_t base = (size_t)b * N;
        if constexpr (Q8) {
            const float inv = 1.0f / l_run;
            float v[4][4], am[2] = {0.f, 0.f};
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int r = 0; r < 4; r += 2) {
                    const unsigned w = pack2<T>(o[dt][r] * inv, o[dt][r + 1] * inv);
                    v[dt][r] = T::to_f32((u16)(w & 0xffff));
                    v[dt][r + 1] = T::to_f32((u16)(w >> 16));
                    am[dt >> 1] = fmaxf(am[dt >> 1], fmaxf(fabsf(v[dt][r]), fabsf(v[dt][r + 1])));
                }
#pragma unroll
            for (int bk = 0; bk < 2; ++bk) {
                am[bk] = fmaxf(am[bk], __shfl_xor(am[bk], 16, 64));
                am[bk] = fmaxf(am[bk], __shfl_xor(am[bk], 32, 64));
            }
            if (q < N) {
                const int e0 = mx_exp(am[0]), e1 = mx_exp(am[1]);
                const float i0 = mx_inv(e0), i1 = mx_inv(e1);
                unsigned char* qrow8 = q8 + (base + q) * D + h * 64;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    const float iv = dt < 2 ? i0 : i1;
                    *(unsigned*)(qrow8 + dt * 16 + 4 * g) =
                        pk4_e4m3(v[dt][0] * iv, v[dt][1] * iv, v[dt][2] * iv, v[dt][3] * iv);
                }
                if (g < 2) q8s[(base + q) * (D / 32) + h * 2 + g] = (unsigned char)((g == 0 ? e0 : e1) + 127);
            }
        } else if (q < N) {
            const float inv = 1.0f / l_run;
            u16* orow = out + (base + q) * D + h * 64;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                uint2 w;
                w.x = pack2<T>(o[dt][0] * inv, o[dt][1] * inv);
                w.y = pack2<T>(o[dt][2] * inv, o[dt][3] * inv);
                *(uint2*)(orow + dt * 16 + 4 * g) = w;
            }
        }
        if (!more) return false;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of stage st done
        __builtin_amdgcn_s_barrier();        // ... every wave's: the unit after next may refill it
        u = un;
        return true;
    };
    while (unit(0, qa, qb) && unit(1, qb, qa)) {
    }
}

// Online-softmax update of one 16-query fragment over a 64-key block (attention_v3, N > 128).
// s holds the raw Q.K scores of the lane's 16 keys (key = kb*64 + 16 kt + 4 g + r). The softmax
// runs in the log2 domain:
// p = exp2(s * c - m), c = log2(e) / sqrt(64), so a score costs one FMA and one v_exp (no
// separate scale multiply, no exp's log2(e) multiply). m_run is kept in that domain. MASK:
// scores with live(kt, r) false become -inf (p = 0); only blocks that can hold dead keys pay it.
// Measured (L/14@336 attention, 24 layers): 9.34 -> 8.70 ms per forward. attention_v2 (B/32) and
// the text tower's kernel keep the scaled-exp form: there it gained nothing, and on the B/32 golden
// fixtures (flat logits) the changed rounding realization raised the worst image 1.38e-3 -> 1.79e-3.
template <bool MASK, typename Live>
__device__ __forceinline__ void softmax_block(f32x4 (&s)[4], float& m_run, float& l_run, f32x4 (&o)[4],
                                              Live&& live) {
    constexpr float c = 0.18033688011112042f;  // log2(e) / 8
    if constexpr (MASK) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (!live(kt, r)) s[kt][r] = -INFINITY;
    }
    float mloc = fmaxf(s[0][0], s[0][1]);  // a chain the compiler folds into v_max3_f32
#pragma unroll
    for (int i = 2; i < 16; ++i) mloc = fmaxf(mloc, s[i >> 2][i & 3]);
    mloc = max_rows4(mloc);
    const float m_new = fmaxf(m_run, mloc * c);
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    m_run = m_new;
    float lsum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float pr = __builtin_amdgcn_exp2f(fmaf(s[kt][r], c, -m_new));
            s[kt][r] = pr;
            lsum += pr;
        }
    l_run = l_run * alpha + lsum;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] *= alpha;
}

// attention_v3_kernel: attention_v2's algorithm with 16 QF queries per wave (QF 16-query
// fragments f; QF = 2; four per wave measured slower in round 1: fewer resident waves). Every K
// fragment (ds_read_b128) and V^T fragment (ds_read_b64_tr_b16) read from LDS feeds two MFMAs instead of one, which halves the LDS read bytes per FLOP: at
// 16 queries per wave v2 reads 32 KB of LDS per 32 MFMAs per SIMD, the LDS array's peak.
// QW waves = 32 QW queries per workgroup; SINGLE as in v2 (N <= 64: one key block, one stage).
template <typename T, int QW = 4, bool SINGLE = false, int QF = 2>
__global__ __launch_bounds__(64 * QW, SINGLE ? 8 : 2) void attention_v3_kernel(const u16* __restrict__ qkv,
                                                                                u16* __restrict__ out, int N, int H) {
    typedef typename T::vec8 vec8;
    constexpr int STAGE = 2 * 64 * 128;  // K [64][128 B] | V [64][128 B]
    __shared__ __attribute__((aligned(16))) unsigned char smem[(SINGLE ? 1 : 2) * STAGE];

    const int D = H * 64;
    const int ld = 3 * D;
    const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 15, g = lane >> 4;
    const size_t base = (size_t)b * N;

    int q[QF];
    vec8 qf[QF][2];
#pragma unroll
    for (int f = 0; f < QF; ++f) {
        q[f] = qb * (16 * QF * QW) + wave * (16 * QF) + f * 16 + j;
        const u16* qrow = qkv + (base + min(q[f], N - 1)) * ld + h * 64;
        qf[f][0] = *(const vec8*)(qrow + 8 * g);
        qf[f][1] = *(const vec8*)(qrow + 32 + 8 * g);
    }

    constexpr int RW = 64 / QW, LPB = 2 * (RW / 8);  // rows per wave, glds per thread per block
    // K/V staging by buffer loads over this image's rows: per-lane offsets constant over the key
    // blocks. The resource is rebased at every key block (base += block offset, range -= block
    // offset: scalar arithmetic), because the hardware range check covers the per-lane offset
    // only, not an SGPR offset. Key rows >= N then lie past the range in every block and read
    // as zeros (their scores are masked, and P = 0 there); nothing past this image's last key row
    // is ever fetched (tests/test_gpu_kernels.py::test_attention_tail_rows_never_read).
    const unsigned char* src = (const unsigned char*)(qkv + base * ld + D + h * 64);
    const unsigned range = (unsigned)((size_t)(N - 1) * ld * 2 + (size_t)D * 2 + 128);
    auto issue = [&](int kb, int st) {
        unsigned char* dst = smem + st * STAGE;
        const unsigned kofs = (unsigned)(kb * 64 * ld * 2);
        const i32x4_t rs = buf_rsrc(src + kofs, range - kofs);
#pragma unroll
        for (int r = 0; r < RW / 8; ++r) {
            const int row = wave * RW + r * 8 + (lane >> 3);
            const int c = (lane & 7) ^ (row & 7);
            const unsigned off = (unsigned)(row * ld * 2 + c * 16);
            blds16(rs, off, 0, dst + (wave * RW + r * 8) * 128);
            blds16(rs, off + (unsigned)D * 2, 0, dst + 8192 + (wave * RW + r * 8) * 128);
        }
    };

    f32x4 o[QF][4];
#pragma unroll
    for (int f = 0; f < QF; ++f)
#pragma unroll
        for (int i = 0; i < 4; ++i) o[f][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m_run[QF], l_run[QF];
#pragma unroll
    for (int f = 0; f < QF; ++f) { m_run[f] = -INFINITY; l_run[f] = 0.f; }
    const int nkb = SINGLE ? 1 : (N + 63) >> 6;

    issue(0, 0);
    if (!SINGLE && nkb > 1) issue(1, 1);
    for (int kb = 0; kb < nkb; ++kb) {
        const int st = kb & 1;
        if (kb + 1 < nkb) vm_wait<LPB>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        const unsigned char* Ks = smem + st * STAGE;
        const unsigned char* Vs = Ks + 8192;

        f32x4 s[QF][4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
#pragma unroll
            for (int f = 0; f < QF; ++f) s[f][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
            const int row = kt * 16 + j;
#pragma unroll
            for (int ds = 0; ds < 2; ++ds) {
                const int c = ((ds << 2) | g) ^ (row & 7);
                const vec8 kf = *(const vec8*)(Ks + row * 128 + (c << 4));
#pragma unroll
                for (int f = 0; f < QF; ++f) s[f][kt] = T::mfma16(kf, qf[f][ds], s[f][kt]);
            }
        }
        auto live = [&](int kt, int r) { return kb * 64 + kt * 16 + 4 * g + r < N; };
        if (kb * 64 + 64 > N) {  // the last block only
#pragma unroll
            for (int f = 0; f < QF; ++f) softmax_block<true>(s[f], m_run[f], l_run[f], o[f], live);
        } else {
#pragma unroll
            for (int f = 0; f < QF; ++f) softmax_block<false>(s[f], m_run[f], l_run[f], o[f], live);
        }

        const int tq = (lane & 15) >> 2, tp = lane & 3;
        const unsigned vbase = (unsigned)(size_t)(LDS_AS const unsigned char*)Vs;
#pragma unroll
        for (int stp = 0; stp < 2; ++stp) {
            u32x2 vr[4][2];
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int hf = 0; hf < 2; ++hf) {
                    const int k = 32 * stp + 16 * hf + 4 * g + tq;
                    const int cl = 2 * dt + (tp >> 1);
                    const unsigned addr = vbase + k * 128 + ((cl ^ (k & 7)) << 4) + 8 * (tp & 1);
                    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(vr[dt][hf]) : "v"(addr) : "memory");
                }
            vec8 pf[QF];
#pragma unroll
            for (int f = 0; f < QF; ++f) {
                unsigned w[4] = {pack2<T>(s[f][2 * stp][0], s[f][2 * stp][1]), pack2<T>(s[f][2 * stp][2], s[f][2 * stp][3]),
                                 pack2<T>(s[f][2 * stp + 1][0], s[f][2 * stp + 1][1]),
                                 pack2<T>(s[f][2 * stp + 1][2], s[f][2 * stp + 1][3])};
                pf[f] = __builtin_bit_cast(vec8, *(uint4*)w);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const uint4 vv = make_uint4(vr[dt][0].x, vr[dt][0].y, vr[dt][1].x, vr[dt][1].y);
#pragma unroll
                for (int f = 0; f < QF; ++f) o[f][dt] = T::mfma16(__builtin_bit_cast(vec8, vv), pf[f], o[f][dt]);
            }
        }
        if (!SINGLE && kb + 2 < nkb) {
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();
            issue(kb + 2, st);
        }
    }

#pragma unroll
    for (int f = 0; f < QF; ++f) {
        float l = l_run[f];
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        if (q[f] < N) {
            const float inv = 1.0f / l;
            u16* orow = out + (base + q[f]) * D + h * 64;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                uint2 w;
                w.x = pack2<T>(o[f][dt][0] * inv, o[f][dt][1] * inv);
                w.y = pack2<T>(o[f][dt][2] * inv, o[f][dt][3] * inv);
                *(uint2*)(orow + dt * 16 + 4 * g) = w;
            }
        }
    }
}

// kernel choice by sequence length: attention_v3 (two query fragments per wave) for N > 128,
// attention_v2 for N <= 128 (one key block at N <= 64: ViT-B/32's N = 50) and for the causal
// text tower (profiles/design_r05.md §11). Two query fragments per wave at N <= 64 measured slower.

// attention with the output quantized to MX-fp8 (q8 [B N, D] e4m3 + q8s [B N, D / 32] scales) in
// the kernel, for the shapes that run on the one-key-block attention_v2 (N <= 64: ViT-B/32);
// returns -1 otherwise (the caller then runs launch_attention + launch_quant_mx8, the same bytes)
// persist > 0: attention_p_kernel on persist workgroups per CU (ncu CUs), else one workgroup per
// (image, head)
static int attn_grid(int units, int persist, int ncu) {
    const int g = persist * (ncu > 0 ? ncu : 256);
    return g < units ? g : units;
}
int launch_attention_q8(hipStream_t s, int dtype, const void* qkv, unsigned char* q8, unsigned char* q8s,
                        int B, int N, int H, int persist, int ncu) {
    if (N > 64) return -1;
    const u16* in = (const u16*)qkv;
    if (persist > 0) {
        const int G = attn_grid(B * H, persist, ncu);
        if (dtype == 2) attention_p_kernel<F16, true><<<G, 256, 0, s>>>(in, nullptr, B, N, H, q8, q8s);
        else attention_p_kernel<BF16, true><<<G, 256, 0, s>>>(in, nullptr, B, N, H, q8, q8s);
        return 0;
    }
    dim3 grid(1, H, B), block(256);
    if (dtype == 2) attention_v2_kernel<F16, 4, true, false, true><<<grid, block, 0, s>>>(in, nullptr, N, H, q8, q8s);
    else attention_v2_kernel<BF16, 4, true, false, true><<<grid, block, 0, s>>>(in, nullptr, N, H, q8, q8s);
    return 0;
}

void launch_attention(hipStream_t s, int dtype, const void* qkv, void* out, int B, int N, int H,
                      bool causal, int persist, int ncu) {
    dim3 grid((N + 63) / 64, H, B), block(256);
    const u16* in = (const u16*)qkv;
    u16* o = (u16*)out;
    if (!causal && N <= 64 && persist > 0) {  // one key block: the persistent loop
        const int G = attn_grid(B * H, persist, ncu);
        if (dtype == 2) attention_p_kernel<F16><<<G, 256, 0, s>>>(in, o, B, N, H);
        else attention_p_kernel<BF16><<<G, 256, 0, s>>>(in, o, B, N, H);
    } else if (causal) {  // text tower: key blocks past the workgroup's last query are skipped
        if (dtype == 2) attention_v2_kernel<F16, 4, false, true><<<grid, block, 0, s>>>(in, o, N, H);
        else attention_v2_kernel<BF16, 4, false, true><<<grid, block, 0, s>>>(in, o, N, H);
    } else if (N > 128) {  // long sequences: 4 waves x 32 queries
        dim3 g4((N + 127) / 128, H, B);
        if (dtype == 2) attention_v3_kernel<F16, 4><<<g4, 256, 0, s>>>(in, o, N, H);
        else attention_v3_kernel<BF16, 4><<<g4, 256, 0, s>>>(in, o, N, H);
    } else if (N <= 64) {  // one key block, one LDS stage
        if (dtype == 2) attention_v2_kernel<F16, 4, true><<<grid, block, 0, s>>>(in, o, N, H);
        else attention_v2_kernel<BF16, 4, true><<<grid, block, 0, s>>>(in, o, N, H);
    } else {
        if (dtype == 2) attention_v2_kernel<F16><<<grid, block, 0, s>>>(in, o, N, H);
        else attention_v2_kernel<BF16><<<grid, block, 0, s>>>(in, o, N, H);
    }
}

}  // namespace clipvit
