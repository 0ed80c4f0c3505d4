// Probe: operand lane map and scale lane map of v_mfma_scale_f32_32x32x64_f8f6f4 (fp8 e4m3)
// on gfx950. The kernel gathers each lane's 32 operand bytes through a host-made table
// (lane, byte) -> k, so several candidate maps are tested in one run; prints PASS/FAIL lines.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/mx32_probe.hip -o /tmp/mx32_probe && /tmp/mx32_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

static float e4m3(unsigned char b) {
    const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
    float v = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + m / 8.f, e - 7);
    return s ? -v : v;
}

// A [32 rows][64 k], B stored [32 cols][64 k]; kmap[l * 32 + j] = k of byte j of lane l.
// Output C[row][col] from the 32x32 C/D map: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
__global__ void probe(const unsigned char* A, const unsigned char* B, const int* kmap, const int* sa,
                      const int* sb, float* C) {
    const int l = threadIdx.x;
    i32x8 a, b;
    unsigned char* pa = (unsigned char*)&a;
    unsigned char* pb = (unsigned char*)&b;
    for (int j = 0; j < 32; ++j) {
        const int k = kmap[l * 32 + j];
        pa[j] = A[(l & 31) * 64 + k];
        pb[j] = B[(l & 31) * 64 + k];
    }
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 0, 0, 0, sa[l], 0, sb[l]);
    for (int r = 0; r < 16; ++r) C[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = acc[r];
}

int main() {
    std::vector<unsigned char> A(32 * 64), B(32 * 64);
    std::vector<float> Af(32 * 64), Bf(32 * 64);
    const unsigned char code[5] = {0xC0, 0xB8, 0x00, 0x38, 0x40};  // -2 -1 0 1 2
    unsigned lcg = 777u;
    auto rnd5 = [&]() { lcg = lcg * 1664525u + 1013904223u; return (int)((lcg >> 16) % 5); };
    for (int i = 0; i < 32 * 64; ++i) {
        const int va = rnd5(), vb = rnd5();
        A[i] = code[va]; Af[i] = (float)(va - 2);
        B[i] = code[vb]; Bf[i] = (float)(vb - 2);
    }
    for (int i = 0; i < 32 * 64; ++i)
        if (e4m3(A[i]) != Af[i] || e4m3(B[i]) != Bf[i]) { printf("FAIL code table\n"); return 1; }
    unsigned char *dA, *dB; int *dk, *dsa, *dsb; float* dC;
    hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dk, 64 * 32 * 4);
    hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dC, 4096);
    hipMemcpy(dA, A.data(), 2048, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 2048, hipMemcpyHostToDevice);

    struct Map { const char* name; int (*k)(int l, int j); };
    const Map maps[] = {
        {"chunks h, h+2 (k = 16h + j | 32 + 16h + j - 16)", [](int l, int j) { const int h = l >> 5; return j < 16 ? 16 * h + j : 32 + 16 * h + (j - 16); }},
        {"contiguous (k = 32h + j)", [](int l, int j) { return 32 * (l >> 5) + j; }},
        {"8-byte pieces (k = 8h + j%8 + 16 (j/8))", [](int l, int j) { return 8 * (l >> 5) + (j & 7) + 16 * (j >> 3); }},
    };
    // scale hypotheses: lane r + 32 b -> row r, k-block b
    int best = -1;
    for (int mi = 0; mi < 3; ++mi) {
        std::vector<int> km(64 * 32);
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 32; ++j) km[l * 32 + j] = maps[mi].k(l, j);
        hipMemcpy(dk, km.data(), km.size() * 4, hipMemcpyHostToDevice);
        bool all = true;
        for (int test = 0; test < 3; ++test) {
            int sa[64], sb[64];
            for (int l = 0; l < 64; ++l) {
                sa[l] = 127; sb[l] = 127;
                if (test == 1) sa[l] = 127 + (l >> 5) + ((l & 31) == 3 ? 2 : 0) + ((l & 31) == 20 ? -1 : 0);
                if (test == 2) sb[l] = 126 + 2 * (l >> 5) + ((l & 31) == 5 ? 1 : 0);
            }
            hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
            hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
            probe<<<1, 64>>>(dA, dB, dk, dsa, dsb, dC);
            float C[1024];
            hipMemcpy(C, dC, 4096, hipMemcpyDeviceToHost);
            double maxerr = 0;
            for (int r = 0; r < 32; ++r)
                for (int c = 0; c < 32; ++c) {
                    double ref = 0;
                    for (int k = 0; k < 64; ++k) {
                        const int kb = k / 32;
                        const double s = std::ldexp(1.0, sa[32 * kb + r] - 127) * std::ldexp(1.0, sb[32 * kb + c] - 127);
                        ref += (double)Af[r * 64 + k] * Bf[c * 64 + k] * s;
                    }
                    maxerr = std::fmax(maxerr, std::fabs(ref - C[r * 32 + c]));
                }
            printf("%s map '%s', scales lane r+32b -> (row r, block b) test %d: max|err| = %g\n",
                   maxerr == 0 ? "PASS" : "FAIL", maps[mi].name, test, maxerr);
            all = all && maxerr == 0;
        }
        if (all && best < 0) best = mi;
    }
    // scale lane scan on the first map: A data nonzero only in k-block KB; raise ONE lane's
    // scale (x2) and list the rows whose outputs changed
    {
        std::vector<int> km(64 * 32);
        const int mi = best < 0 ? 0 : best;
        for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 32; ++j) km[l * 32 + j] = maps[mi].k(l, j);
        hipMemcpy(dk, km.data(), km.size() * 4, hipMemcpyHostToDevice);
        for (int KB = 0; KB < 2; ++KB) {
            std::vector<unsigned char> A2(A);
            for (int r = 0; r < 32; ++r)
                for (int k = 0; k < 64; ++k)
                    if (k / 32 != KB) A2[r * 64 + k] = 0;
            hipMemcpy(dA, A2.data(), 2048, hipMemcpyHostToDevice);
            int sa[64], sb[64];
            for (int l = 0; l < 64; ++l) sa[l] = sb[l] = 127;
            hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
            hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
            float Cb[1024];
            probe<<<1, 64>>>(dA, dB, dk, dsa, dsb, dC);
            hipMemcpy(Cb, dC, 4096, hipMemcpyDeviceToHost);
            printf("A scale scan KB%d:", KB);
            for (int L = 0; L < 64; ++L) {
                for (int l = 0; l < 64; ++l) sa[l] = 127;
                sa[L] = 128;
                hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
                float C[1024];
                probe<<<1, 64>>>(dA, dB, dk, dsa, dsb, dC);
                hipMemcpy(C, dC, 4096, hipMemcpyDeviceToHost);
                std::string d;
                for (int r = 0; r < 32; ++r) {
                    double num = 0, den = 0;
                    for (int c = 0; c < 32; ++c) { num += std::fabs(C[r * 32 + c]); den += std::fabs(Cb[r * 32 + c]); }
                    if (std::fabs(num - den) > 1e-3 * (den + 1)) d += " " + std::to_string(r);
                }
                if (!d.empty()) printf(" L%d(%s)", L, d.c_str());
            }
            printf("\n");
        }
    }
    printf("best map: %d\n", best);
    return 0;
}
