// Probe: operand lane map and scale semantics of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3)
// and the byte encoding of v_cvt_pk_fp8_f32 on gfx950. Prints PASS/FAIL lines.
//   hipcc --offload-arch=gfx950 -O2 tools/probes/mx_probe.hip -o /tmp/mx_probe && /tmp/mx_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
#include <string>
#include <utility>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// e4m3 (OCP) decode on the host
static float e4m3(unsigned char b) {
    const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
    float v = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + m / 8.f, e - 7);
    if (e == 15 && m == 7) v = NAN;
    return s ? -v : v;
}

__global__ void mfma_probe(const unsigned char* A, const unsigned char* B, const int* sa,
                           const int* sb, float* C) {
    const int l = threadIdx.x;
    // measured map: lane l (g = l >> 4) holds A[l & 15][k] with k = 16 g + j for bytes j < 16
    // and k = 64 + 16 g + (j - 16) for bytes j >= 16 (two stacked 16x16x64 halves); the
    // E8M0 scale of lane r + 16 b applies to row r, k-block b = k / 32 (same for B / cols)
    i32x8 a, b;
    unsigned char* pa = (unsigned char*)&a;
    unsigned char* pb = (unsigned char*)&b;
    const int g = l >> 4;
    for (int j = 0; j < 32; ++j) {
        const int k = j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16);
        pa[j] = A[(l & 15) * 128 + k];
        pb[j] = B[(l & 15) * 128 + k];  // B stored as [col][k]
    }
    f32x4 acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa[l], 0, sb[l]);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];  // row, col
}

__global__ void cvt_probe(const float* x, unsigned* o, int n) {
    const int i = threadIdx.x;
    if (2 * i + 1 < n) o[i] = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
}

int main() {
    // conversion
    const float xs[8] = {1.f, -2.f, 448.f, 0.0625f, 3.3f, -0.01953125f, 500.f, 1.0e-4f};
    float* dx; unsigned* dout;
    hipMalloc(&dx, sizeof(xs)); hipMalloc(&dout, 16);
    hipMemcpy(dx, xs, sizeof(xs), hipMemcpyHostToDevice);
    cvt_probe<<<1, 4>>>(dx, dout, 8);
    unsigned ob[4];
    hipMemcpy(ob, dout, 16, hipMemcpyDeviceToHost);
    printf("cvt bytes:");
    for (int i = 0; i < 8; ++i) {
        const unsigned char b = (ob[i / 2] >> (8 * (i & 1))) & 0xff;
        printf(" %g->0x%02x(%g)", xs[i], b, e4m3(b));
    }
    printf("\n");
    const bool cvt_ok = ((ob[0] & 0xff) == 0x38) && (((ob[0] >> 8) & 0xff) == 0xC0) && ((ob[1] & 0xff) == 0x7E);
    printf("%s cvt_pk_fp8_f32 OCP e4m3 (1.0=0x38, -2=0xC0, 448=0x7E), lo byte = first operand\n",
           cvt_ok ? "PASS" : "FAIL");

    // MFMA: A [16][128], B stored [16 cols][128 k], small exact integers
    std::vector<unsigned char> A(16 * 128), B(16 * 128);
    std::vector<float> Af(16 * 128), Bf(16 * 128);
    // e4m3 codes for small integers: 0->0x00, 1->0x38, 2->0x40, 3->0x44, -1->0xB8, -2->0xC0
    const unsigned char code[5] = {0xC0, 0xB8, 0x00, 0x38, 0x40};
    unsigned lcg = 12345u;
    auto rnd5 = [&]() { lcg = lcg * 1664525u + 1013904223u; return (int)((lcg >> 16) % 5); };
    for (int i = 0; i < 16 * 128; ++i) {
        const int va = rnd5(), vb = rnd5();
        A[i] = code[va]; Af[i] = (float)(va - 2);
        B[i] = code[vb]; Bf[i] = (float)(vb - 2);
    }
    unsigned char *dA, *dB; int *dsa, *dsb; float* dC;
    hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256);
    hipMalloc(&dC, 1024);
    hipMemcpy(dA, A.data(), 2048, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 2048, hipMemcpyHostToDevice);
    for (int test = 0; test < 3; ++test) {
        int sa[64], sb[64];
        for (int l = 0; l < 64; ++l) {
            sa[l] = 127; sb[l] = 127;
            if (test == 1) sa[l] = 127 + (l >> 4) + ((l & 15) == 3 ? 2 : 0);  // per (row, k-block)
            if (test == 2) sb[l] = 126 + (l >> 4) + ((l & 15) == 5 ? 1 : 0);  // per (col, k-block)
        }
        hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
        hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
        mfma_probe<<<1, 64>>>(dA, dB, dsa, dsb, dC);
        float C[256];
        hipMemcpy(C, dC, 1024, hipMemcpyDeviceToHost);
        double maxerr = 0;
        for (int r = 0; r < 16; ++r)
            for (int c = 0; c < 16; ++c) {
                double ref = 0;
                for (int k = 0; k < 128; ++k) {
                    const int kb = k / 32;
                    // scale of A row r, block kb is held by lane 16*kb + r; of B col c by lane 16*kb + c
                    const double s = std::ldexp(1.0, sa[16 * kb + r] - 127) * std::ldexp(1.0, sb[16 * kb + c] - 127);
                    ref += (double)Af[r * 128 + k] * Bf[c * 128 + k] * s;
                }
                maxerr = std::fmax(maxerr, std::fabs(ref - C[r * 16 + c]));
            }
        printf("%s mfma_scale 16x16x128 fp8 lane map + scales (test %d): max|err| = %g\n",
               maxerr == 0 ? "PASS" : "FAIL", test, maxerr);
    }
    hipMemcpy(dB, B.data(), 2048, hipMemcpyHostToDevice);
    for (int test = 0; test < 3; ++test) {
        int sa[64], sb[64];
        for (int l = 0; l < 64; ++l) {
            sa[l] = 127; sb[l] = 127;
            if (test == 1) sa[l] = 127 + (l >> 4) + ((l & 15) == 3 ? 2 : 0);  // per (row, k-block)
            if (test == 2) sb[l] = 126 + (l >> 4) + ((l & 15) == 5 ? 1 : 0);  // per (col, k-block)
        }
        hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
        hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
        mfma_probe<<<1, 64>>>(dA, dB, dsa, dsb, dC);
        float C[256];
        hipMemcpy(C, dC, 1024, hipMemcpyDeviceToHost);
        double maxerr = 0;
        for (int r = 0; r < 16; ++r)
            for (int c = 0; c < 16; ++c) {
                double ref = 0;
                for (int k = 0; k < 128; ++k) {
                    const int kb = k / 32;
                    // scale of A row r, block kb is held by lane 16*kb + r; of B col c by lane 16*kb + c
                    const double s = std::ldexp(1.0, sa[16 * kb + r] - 127) * std::ldexp(1.0, sb[16 * kb + c] - 127);
                    ref += (double)Af[r * 128 + k] * Bf[c * 128 + k] * s;
                }
                maxerr = std::fmax(maxerr, std::fabs(ref - C[r * 16 + c]));
            }
        printf("%s mfma_scale 16x16x128 fp8 lane map + scales (test %d): max|err| = %g\n",
               maxerr == 0 ? "PASS" : "FAIL", test, maxerr);
    }
    // scale lane map: A data nonzero only in k-block KB; raise ONE lane's scale by 1 (x2) and
    // report the rows whose outputs changed and the ratio new/base (2 = full control).
    for (int which = 0; which < 2; ++which) {
        printf("%s scale lane -> (row|col: ratio) per k-block\n", which ? "B" : "A");
        for (int KB = 0; KB < 4; ++KB) {
            std::vector<unsigned char> A2(A);
            for (int r = 0; r < 16; ++r)
                for (int k = 0; k < 128; ++k)
                    if (k / 32 != KB) A2[r * 128 + k] = 0;
            hipMemcpy(dA, A2.data(), 2048, hipMemcpyHostToDevice);
            int sa[64], sb[64];
            for (int l = 0; l < 64; ++l) sa[l] = sb[l] = 127;
            hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
            hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
            float Cb[256];
            mfma_probe<<<1, 64>>>(dA, dB, dsa, dsb, dC);
            hipMemcpy(Cb, dC, 1024, hipMemcpyDeviceToHost);
            printf(" KB%d:", KB);
            for (int L = 0; L < 64; ++L) {
                for (int l = 0; l < 64; ++l) sa[l] = sb[l] = 127;
                (which ? sb : sa)[L] = 128;
                hipMemcpy(dsa, sa, 256, hipMemcpyHostToDevice);
                hipMemcpy(dsb, sb, 256, hipMemcpyHostToDevice);
                float C[256];
                mfma_probe<<<1, 64>>>(dA, dB, dsa, dsb, dC);
                hipMemcpy(C, dC, 1024, hipMemcpyDeviceToHost);
                std::string d;
                for (int rc = 0; rc < 16; ++rc) {
                    double num = 0, den = 0;
                    for (int o = 0; o < 16; ++o) {
                        const int r = which ? o : rc, c = which ? rc : o;
                        num += std::fabs(C[r * 16 + c]); den += std::fabs(Cb[r * 16 + c]);
                    }
                    if (std::fabs(num - den) > 1e-3 * (den + 1)) {
                        char buf[48];
                        snprintf(buf, sizeof buf, "%d:%.2f", rc, num / den);
                        d += buf;
                    }
                }
                if (!d.empty()) printf(" L%d(%s)", L, d.c_str());
            }
            printf("\n");
        }
    }
    hipMemcpy(dA, A.data(), 2048, hipMemcpyHostToDevice);
    return 0;
}
