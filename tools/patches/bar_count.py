"""Diagnostic (never in the product): every row-stream step barrier counts itself per (workgroup, wave) in a buffer set by
psgla_barcount_set() (tools/bar_probe.py), so a launch's per-wave barrier counts can be compared."""
PATCHES = [
    ("__device__ __forceinline__ void step_barrier() { lds_barrier(); }",
     """static __device__ int* g_barcount = nullptr;
__device__ __forceinline__ void step_barrier() {
    if ((threadIdx.x & 63) == 0 && g_barcount)
        __hip_atomic_fetch_add(g_barcount + blockIdx.x * 16 + (threadIdx.x >> 6), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lds_barrier();
}""", 1),
    ("void launch_stream(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen, bool half) {",
     """extern "C" int psgla_barcount_set(void* p) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_barcount), &p, sizeof(p)); }
void launch_stream(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen, bool half) {""", 1),
]
FORCE = ["tv_stream.hip"]
