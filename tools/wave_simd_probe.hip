// Which SIMD each wave of a 16-wave workgroup runs on (diagnostic): HW_ID bits 5:4 (SIMD), 11:8 (CU).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/wave_simd_probe tools/wave_simd_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(1024) void probe(unsigned* out) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = hw;
}
int main() {
    unsigned* d;
    hipMalloc(&d, 4 * 16 * 4);
    hipLaunchKernelGGL(probe, dim3(4), dim3(1024), 0, 0, d);
    unsigned h[64];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int b = 0; b < 4; ++b) {
        printf("wg %d simd of waves 0..15:", b);
        for (int w = 0; w < 16; ++w) printf(" %u", (h[b * 16 + w] >> 4) & 3);
        printf("   (wave slot:");
        for (int w = 0; w < 16; ++w) printf(" %u", h[b * 16 + w] & 15);
        printf(")\n");
    }
    return 0;
}
