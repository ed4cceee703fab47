// VALU issue-rate probe for gfx950 (diagnostic, never in the product library).
//
// One workgroup per CU (grid = 256) of 64 x 4 x WPS threads, i.e. WPS waves on each of the CU's 4 SIMDs.  Every wave
// runs ITERS iterations of 8 copies of a block of 16 independent VALU instructions (16 accumulators, no dependent
// pair closer than 16 instructions; 128 instructions per loop branch) and stamps the shader clock (s_memtime) around the loop.  Reported: SIMD cycles per
// wave-instruction = wave cycles / (16 ITERS WPS) -- 2 means two waves' instructions overlap, 4 that the SIMD
// issues one wave64 instruction per 4 cycles whatever the number of waves.
//
// The forms differ in operand sources, to find what the tile / stream kernels' iteration loops pay:
//   fma3v       v_fma_f32 acc, vA, vB, acc    three VGPR sources, banks spread (acc banks 0/3, vA 1, vB 2)
//   fma3v_same  v_fma_f32 acc, vA, vB, acc    three VGPR sources, all in bank 0
//   fma_s       v_fma_f32 acc, sK, vB, acc    one SGPR source
//   fmac        v_fmac_f32 acc, vA, vB        VOP2 (acc read as the addend)
//   add         v_add_f32 acc, vA, acc
//   sub_2v      v_sub_f32 acc, vA, vB         two sources, result not read by the block
//   rsq         v_rsq_f32 acc, vA
//   mix         the tile iteration's mix: 6 sub, 6 fma (VOP3), 4 fmac, 3 mul, 1 rsq, 1 min per 21
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/valu_probe tools/valu_probe.hip; run: tools/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CLOBBERS                                                                                                 \
    "v1", "v2", "v4", "v8", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43",  \
        "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", \
        "v59", "v60", "v61", "v62", "v63"

#define INIT_ASM                                                                                                 \
    "v_mov_b32 v1, 1.0\n v_mov_b32 v2, 0.5\n v_mov_b32 v4, 1.0\n v_mov_b32 v8, 0.5\n"                           \
    "v_mov_b32 v32, 0\n v_mov_b32 v35, 0\n v_mov_b32 v36, 0\n v_mov_b32 v39, 0\n"                                \
    "v_mov_b32 v40, 0\n v_mov_b32 v43, 0\n v_mov_b32 v44, 0\n v_mov_b32 v47, 0\n"                                \
    "v_mov_b32 v48, 0\n v_mov_b32 v51, 0\n v_mov_b32 v52, 0\n v_mov_b32 v55, 0\n"                                \
    "v_mov_b32 v56, 0\n v_mov_b32 v59, 0\n v_mov_b32 v60, 0\n v_mov_b32 v63, 0\n"

#define BODY_fma3v                                                                                               \
    "v_fma_f32 v32, v1, v2, v32\n v_fma_f32 v35, v1, v2, v35\n v_fma_f32 v36, v1, v2, v36\n v_fma_f32 v39, v1, v2, v39\n" \
    "v_fma_f32 v40, v1, v2, v40\n v_fma_f32 v43, v1, v2, v43\n v_fma_f32 v44, v1, v2, v44\n v_fma_f32 v47, v1, v2, v47\n" \
    "v_fma_f32 v48, v1, v2, v48\n v_fma_f32 v51, v1, v2, v51\n v_fma_f32 v52, v1, v2, v52\n v_fma_f32 v55, v1, v2, v55\n" \
    "v_fma_f32 v56, v1, v2, v56\n v_fma_f32 v59, v1, v2, v59\n v_fma_f32 v60, v1, v2, v60\n v_fma_f32 v63, v1, v2, v63\n"
#define BODY_fma3v_same                                                                                          \
    "v_fma_f32 v32, v4, v8, v32\n v_fma_f32 v36, v4, v8, v36\n v_fma_f32 v40, v4, v8, v40\n v_fma_f32 v44, v4, v8, v44\n" \
    "v_fma_f32 v48, v4, v8, v48\n v_fma_f32 v52, v4, v8, v52\n v_fma_f32 v56, v4, v8, v56\n v_fma_f32 v60, v4, v8, v60\n" \
    "v_fma_f32 v32, v4, v8, v32\n v_fma_f32 v36, v4, v8, v36\n v_fma_f32 v40, v4, v8, v40\n v_fma_f32 v44, v4, v8, v44\n" \
    "v_fma_f32 v48, v4, v8, v48\n v_fma_f32 v52, v4, v8, v52\n v_fma_f32 v56, v4, v8, v56\n v_fma_f32 v60, v4, v8, v60\n"
#define BODY_fma_s                                                                                               \
    "v_fma_f32 v32, %1, v2, v32\n v_fma_f32 v35, %1, v2, v35\n v_fma_f32 v36, %1, v2, v36\n v_fma_f32 v39, %1, v2, v39\n" \
    "v_fma_f32 v40, %1, v2, v40\n v_fma_f32 v43, %1, v2, v43\n v_fma_f32 v44, %1, v2, v44\n v_fma_f32 v47, %1, v2, v47\n" \
    "v_fma_f32 v48, %1, v2, v48\n v_fma_f32 v51, %1, v2, v51\n v_fma_f32 v52, %1, v2, v52\n v_fma_f32 v55, %1, v2, v55\n" \
    "v_fma_f32 v56, %1, v2, v56\n v_fma_f32 v59, %1, v2, v59\n v_fma_f32 v60, %1, v2, v60\n v_fma_f32 v63, %1, v2, v63\n"
#define BODY_fmac                                                                                                \
    "v_fmac_f32 v32, v1, v2\n v_fmac_f32 v35, v1, v2\n v_fmac_f32 v36, v1, v2\n v_fmac_f32 v39, v1, v2\n"         \
    "v_fmac_f32 v40, v1, v2\n v_fmac_f32 v43, v1, v2\n v_fmac_f32 v44, v1, v2\n v_fmac_f32 v47, v1, v2\n"         \
    "v_fmac_f32 v48, v1, v2\n v_fmac_f32 v51, v1, v2\n v_fmac_f32 v52, v1, v2\n v_fmac_f32 v55, v1, v2\n"         \
    "v_fmac_f32 v56, v1, v2\n v_fmac_f32 v59, v1, v2\n v_fmac_f32 v60, v1, v2\n v_fmac_f32 v63, v1, v2\n"
#define BODY_add                                                                                                 \
    "v_add_f32 v32, v1, v32\n v_add_f32 v35, v1, v35\n v_add_f32 v36, v1, v36\n v_add_f32 v39, v1, v39\n"         \
    "v_add_f32 v40, v1, v40\n v_add_f32 v43, v1, v43\n v_add_f32 v44, v1, v44\n v_add_f32 v47, v1, v47\n"         \
    "v_add_f32 v48, v1, v48\n v_add_f32 v51, v1, v51\n v_add_f32 v52, v1, v52\n v_add_f32 v55, v1, v55\n"         \
    "v_add_f32 v56, v1, v56\n v_add_f32 v59, v1, v59\n v_add_f32 v60, v1, v60\n v_add_f32 v63, v1, v63\n"
#define BODY_sub_2v                                                                                              \
    "v_sub_f32 v32, v1, v2\n v_sub_f32 v35, v1, v2\n v_sub_f32 v36, v1, v2\n v_sub_f32 v39, v1, v2\n"             \
    "v_sub_f32 v40, v1, v2\n v_sub_f32 v43, v1, v2\n v_sub_f32 v44, v1, v2\n v_sub_f32 v47, v1, v2\n"             \
    "v_sub_f32 v48, v1, v2\n v_sub_f32 v51, v1, v2\n v_sub_f32 v52, v1, v2\n v_sub_f32 v55, v1, v2\n"             \
    "v_sub_f32 v56, v1, v2\n v_sub_f32 v59, v1, v2\n v_sub_f32 v60, v1, v2\n v_sub_f32 v63, v1, v2\n"
#define BODY_rsq                                                                                                 \
    "v_rsq_f32 v32, v1\n v_rsq_f32 v35, v1\n v_rsq_f32 v36, v1\n v_rsq_f32 v39, v1\n"                             \
    "v_rsq_f32 v40, v1\n v_rsq_f32 v43, v1\n v_rsq_f32 v44, v1\n v_rsq_f32 v47, v1\n"                             \
    "v_rsq_f32 v48, v1\n v_rsq_f32 v51, v1\n v_rsq_f32 v52, v1\n v_rsq_f32 v55, v1\n"                             \
    "v_rsq_f32 v56, v1\n v_rsq_f32 v59, v1\n v_rsq_f32 v60, v1\n v_rsq_f32 v63, v1\n"
// 21 instructions in the tile loop's proportions (6 sub, 6 fma, 4 fmac, 3 mul, 1 rsq, 1 min); counted as 21
#define BODY_mix                                                                                                 \
    "v_sub_f32 v32, v1, v2\n v_fma_f32 v35, %1, v2, v35\n v_sub_f32 v36, v39, v2\n v_fmac_f32 v40, v1, v2\n"      \
    "v_mul_f32 v43, v1, v43\n v_fma_f32 v44, v47, v2, v44\n v_sub_f32 v48, v1, v51\n v_fma_f32 v52, %1, v55, v52\n" \
    "v_rsq_f32 v56, v1\n v_sub_f32 v59, v60, v2\n v_fmac_f32 v63, v1, v2\n v_fma_f32 v32, v35, v36, v32\n"        \
    "v_mul_f32 v39, v1, v39\n v_sub_f32 v40, v43, v44\n v_fma_f32 v47, %1, v48, v47\n v_min_f32 v51, 1.0, v51\n"  \
    "v_fmac_f32 v55, v56, v2\n v_sub_f32 v59, v1, v63\n v_fma_f32 v60, v1, v2, v60\n v_mul_f32 v35, v1, v35\n"     \
    "v_fmac_f32 v36, v1, v2\n"

#define PROBE(NAME, NINST)                                                                                        \
    __global__ __launch_bounds__(1024) void probe_##NAME(unsigned long long* out, int iters, float s) {          \
        asm volatile(INIT_ASM ::: CLOBBERS);                                                                      \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                               \
        for (int i = 0; i < iters; ++i) {                                                                         \
            asm volatile(BODY_##NAME BODY_##NAME BODY_##NAME BODY_##NAME BODY_##NAME BODY_##NAME BODY_##NAME BODY_##NAME : "+s"(i) : "s"(s) : CLOBBERS);                                              \
        }                                                                                                         \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                               \
        float r;                                                                                                  \
        asm volatile("v_add_f32 %0, v32, v35" : "=v"(r) :: CLOBBERS);                                             \
        if ((threadIdx.x & 63) == 0) {                                                                            \
            const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;                                        \
            out[2 * wave] = t1 - t0;                                                                              \
            out[2 * wave + 1] = (unsigned long long)(r == 12345.f);                                              \
        }                                                                                                         \
    }                                                                                                             \
    static const int kInst_##NAME = NINST;

PROBE(fma3v, 16)
PROBE(fma3v_same, 16)
PROBE(fma_s, 16)
PROBE(fmac, 16)
PROBE(add, 16)
PROBE(sub_2v, 16)
PROBE(rsq, 16)
PROBE(mix, 21)

#define CHECK(x)                                                                                                  \
    do {                                                                                                          \
        hipError_t e_ = (x);                                                                                      \
        if (e_ != hipSuccess) {                                                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                               \
            exit(1);                                                                                              \
        }                                                                                                         \
    } while (0)

template <typename K>
static void run(const char* name, K kern, int ninst, int wps, unsigned long long* d_out) {
    const int grid = 256, threads = 64 * 4 * wps, iters = 500;
    const int waves = grid * threads / 64;
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, d_out, iters, 0.5f);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, d_out, iters, 0.5f);
    CHECK(hipEventRecord(e1));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(2 * waves);
    CHECK(hipMemcpy(h.data(), d_out, h.size() * 8, hipMemcpyDeviceToHost));
    double mean = 0, mx = 0;
    for (int w = 0; w < waves; ++w) {
        mean += (double)h[2 * w];
        if ((double)h[2 * w] > mx) mx = (double)h[2 * w];
    }
    mean /= waves;
    const double inst = (double)ninst * 8 * iters;   // 8 copies of the block per loop iteration
    printf("%-11s waves/SIMD %d | wave cycles per instruction %6.2f | SIMD cycles per wave-instruction %5.2f (max wave %5.2f) | kernel %.3f ms\n",
           name, wps, mean / inst, mean / (inst * wps), mx / (inst * wps), ms);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

int main() {
    unsigned long long* d_out;
    CHECK(hipMalloc(&d_out, 2 * 256 * 16 * 8));
#define RUN(NAME)                                                                                                 \
    for (int wps : {1, 2, 4}) run(#NAME, probe_##NAME, kInst_##NAME, wps, d_out);
    RUN(fma3v)
    RUN(fma3v_same)
    RUN(fma_s)
    RUN(fmac)
    RUN(add)
    RUN(sub_2v)
    RUN(rsq)
    RUN(mix)
    CHECK(hipFree(d_out));
    return 0;
}
