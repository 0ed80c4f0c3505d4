// Probe: which XCDs / CUs run the workgroups of a kernel launched on a CU-masked stream
// (hipExtStreamCreateWithCUMask). Each workgroup writes its XCC_ID and HW_ID (vector store).
//   hipcc --offload-arch=gfx950 -O2 tools/probes/cumask_probe.hip -o /tmp/cumask_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <set>

__global__ void whereami(unsigned* out) {
    // lanes 0 and 1 write (vector stores: the value and address depend on the lane)
    const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID (id 20), bits [3:0]
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID (id 4)
    if (threadIdx.x < 2) out[2 * blockIdx.x + threadIdx.x] = threadIdx.x == 0 ? xcc : hw;
    // keep the workgroup resident a little so the dispatcher spreads the grid
    for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(1);
}

static void run(const char* tag, const std::vector<uint32_t>& mask) {
    hipStream_t s;
    if (mask.empty()) hipStreamCreate(&s);
    else if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) { printf("%s: mask refused\n", tag); return; }
    const int nb = 2048;
    unsigned* d;
    hipMalloc(&d, nb * 2 * sizeof(unsigned));
    hipLaunchKernelGGL(whereami, dim3(nb), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    std::vector<unsigned> h(nb * 2);
    hipMemcpy(h.data(), d, nb * 2 * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::set<unsigned> xcds; std::set<unsigned> cus[8];
    int per[8] = {0};
    for (int b = 0; b < nb; ++b) {
        const unsigned x = h[2 * b] & 15, hw = h[2 * b + 1];
        xcds.insert(x);
        // HW_ID: cu_id [11:8], sh_id [12], se_id [15:13] (gfx9 layout)
        cus[x & 7].insert(((hw >> 13) & 7) * 32 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15));
        per[x & 7]++;
    }
    printf("%-28s xcds used:", tag);
    for (unsigned x : xcds) printf(" %u", x);
    printf(" | blocks per xcd:");
    for (int i = 0; i < 8; ++i) printf(" %d", per[i]);
    printf(" | distinct CUs per xcd:");
    for (int i = 0; i < 8; ++i) printf(" %zu", cus[i].size());
    printf(" | first blocks' xcd:");
    for (int b = 0; b < 16; ++b) printf(" %u", h[2 * b] & 15);
    printf("\n");
    hipFree(d);
    hipStreamDestroy(s);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("CUs %d\n", p.multiProcessorCount);
    run("no mask", {});
    std::vector<uint32_t> lo(8, 0), hi(8, 0), even(8, 0), quarter(8, 0);
    for (int i = 0; i < 4; ++i) lo[i] = 0xffffffffu;        // bits 0..127
    for (int i = 4; i < 8; ++i) hi[i] = 0xffffffffu;        // bits 128..255
    for (int i = 0; i < 8; ++i) even[i] = 0x55555555u;      // every other bit
    quarter[0] = 0xffffffffu;                                // bits 0..31
    run("bits 0-127", lo);
    run("bits 128-255", hi);
    run("even bits", even);
    run("bits 0-31", quarter);
    std::vector<uint32_t> m8(8, 0);
    for (int i = 0; i < 8; ++i) m8[i] = 0x01010101u;         // bits 0, 8, 16, ...
    run("bits 0,8,16,...", m8);
    // XCD-set masks, if mask bit i maps to XCD i % 8: bits with i % 8 < 4 / >= 4
    std::vector<uint32_t> x03(8, 0x0f0f0f0fu), x47(8, 0xf0f0f0f0u);
    run("bits i%8<4", x03);
    run("bits i%8>=4", x47);
    // XCD-set masks, if bit i maps to XCD i / 32: words 0-3 / 4-7 (= bits 0-127 / 128-255 above)
    return 0;
}
