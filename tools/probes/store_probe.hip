// Epilogue-store probe (profiles/design_r05.md §5.8): how fast can 256 workgroups (one per CU, 8 waves) write
// 16-bit 256x256 output tiles, by lane->address pattern? Same bytes in every arm.
//
//   frag : the ping-pong GEMM's pattern: for fm in 0..7 a wave stores rows (16 per fm) x 64 features,
//          lane (r, g) = 32 B of row r at features 16 g .. 16 g + 15 (two dwordx4 per lane)
//   rowc : the same 16 rows x 128 B per fm, but each store instruction covers 8 whole rows
//          (lane -> row lane >> 3, 16-B chunk lane & 7): full 128-B lines per quarter-wave
//   *_nt : the same with non-temporal stores
// Grid: `tiles` tiles walked persistently by 256 workgroups (c_fc at bs 256: 600 tiles of
// 12800 x 3072); optional `spin` = s_sleep units between tiles (compute stand-in).
//
// hipcc --offload-arch=gfx950 -O3 -o tools/probes/store_probe tools/probes/store_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int PAT, bool NT>
__global__ __launch_bounds__(512, 1) void store_kernel(unsigned short* C, int M, int N, int ntiles, int spin) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = wave >> 2, wc = wave & 3;
    const int nN = N / 256;
    unsigned char* Cb = (unsigned char*)C;
    const u32x4 val = {(unsigned)lane, (unsigned)wave, 0x3c003c00u, (unsigned)blockIdx.x};
    for (int L = blockIdx.x; L < ntiles; L += gridDim.x) {
        const int mt = L / nN, nt = L % nN;
        const int m0 = mt * 256, n0 = nt * 256;
#pragma unroll
        for (int fm = 0; fm < 8; ++fm) {
            if constexpr (PAT == 0) {
                const int m = m0 + grp * 128 + fm * 16 + (lane & 15);
                const int n = n0 + wc * 64 + 16 * (lane >> 4);
                const size_t off = ((size_t)m * N + n) * 2;
                if (NT) {
                    __builtin_nontemporal_store(val, (u32x4*)(Cb + off));
                    __builtin_nontemporal_store(val, (u32x4*)(Cb + off + 16));
                } else {
                    *(u32x4*)(Cb + off) = val;
                    *(u32x4*)(Cb + off + 16) = val;
                }
            } else if constexpr (PAT == 2) {  // "half": lanes r, r ^ 8 swap halves: 8 rows x 32 B per quarter-wave
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int r = lane & 15, g = lane >> 4;
                    const int m = m0 + grp * 128 + fm * 16 + i * 8 + (r & 7);
                    const int n = n0 + wc * 64 + 8 * (2 * g + (r >> 3));
                    const size_t off = ((size_t)m * N + n) * 2;
                    *(u32x4*)(Cb + off) = val;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int m = m0 + grp * 128 + fm * 16 + i * 8 + (lane >> 3);
                    const int n = n0 + wc * 64 + 8 * (lane & 7);
                    const size_t off = ((size_t)m * N + n) * 2;
                    if (NT) __builtin_nontemporal_store(val, (u32x4*)(Cb + off));
                    else *(u32x4*)(Cb + off) = val;
                }
            }
        }
        for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(127);
    }
}

template <int PAT, bool NT>
static float run(unsigned short* C, int M, int N, int ntiles, int spin, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = ntiles < 256 ? ntiles : 256;
    store_kernel<PAT, NT><<<grid, 512>>>(C, M, N, ntiles, spin);
    hipEventRecord(a);
    for (int i = 0; i < iters; ++i) store_kernel<PAT, NT><<<grid, 512>>>(C, M, N, ntiles, spin);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return ms * 1e3f / iters;
}

int main(int argc, char** argv) {
    const int M = 12800, N = 3072;
    unsigned short* C = nullptr;
    if (hipMalloc(&C, (size_t)M * N * 2) != hipSuccess) return 1;
    // one tile per workgroup on 8 .. 256 CUs: per-CU store time vs chip-wide burst
    for (int nt : {8, 32, 64, 128, 256}) {
        float t0 = 1e9f, t1 = 1e9f, t2 = 1e9f;
        for (int r = 0; r < 3; ++r) {
            t0 = fminf(t0, run<0, false>(C, M, N, nt, 0, 20));
            t1 = fminf(t1, run<1, false>(C, M, N, nt, 0, 20));
            t2 = fminf(t2, run<2, false>(C, M, N, nt, 0, 20));
        }
        printf("grid %3d (one tile each): frag %.2f us  rowc %.2f us  half %.2f us\n", nt, t0, t1, t2);
    }
    for (int nt : {512, 600}) {
        float t0 = 1e9f, t1 = 1e9f, t2 = 1e9f;
        for (int r = 0; r < 3; ++r) {
            t0 = fminf(t0, run<0, false>(C, M, N, nt, 0, 20));
            t1 = fminf(t1, run<1, false>(C, M, N, nt, 0, 20));
            t2 = fminf(t2, run<2, false>(C, M, N, nt, 0, 20));
        }
        printf("tiles %3d: frag %.2f us  rowc %.2f us  half %.2f us\n", nt, t0, t1, t2);
    }
    const int tile_sets[3] = {256, 512, 600};
    for (int spin : {0}) {
        for (int nt : tile_sets) {
            float t[4] = {};
            for (int r = 0; r < 3; ++r) {  // interleaved rounds; keep the min
                const float f0 = run<0, false>(C, M, N, nt, spin, 20), f1 = run<1, false>(C, M, N, nt, spin, 20);
                const float f2 = run<0, true>(C, M, N, nt, spin, 20), f3 = run<1, true>(C, M, N, nt, spin, 20);
                const float v[4] = {f0, f1, f2, f3};
                for (int k = 0; k < 4; ++k) t[k] = r == 0 || v[k] < t[k] ? v[k] : t[k];
            }
            const double mb = (double)nt * 256 * 256 * 2 / 1e6;
            printf("tiles %3d spin %d (%.1f MB): frag %.1f us (%.2f TB/s)  rowc %.1f us (%.2f)  frag_nt %.1f (%.2f)  rowc_nt %.1f (%.2f)\n",
                   nt, spin, mb, t[0], mb / t[0], t[1], mb / t[1], t[2], mb / t[2], t[3], mb / t[3]);
        }
    }
    hipFree(C);
    return 0;
}
