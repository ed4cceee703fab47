"""Diagnostic (never in the product): every inline-asm global access of the library (LDS-DMA loads, nt / sc1 stores) checks
its address first; an address outside [64 KiB, 2^47) is skipped and recorded in a buffer set by psgla_guard_set():
[0] count, [1 + 64 * prim + wave] the last bad address (prim 0 glds16, 1 glds16_at, 2 glds4, 3 st_nt, 4 st_tile),
[400] the last launch step read at kernel start that was outside [0, 2^31) (tools/guard_probe.py)."""
GUARD = r'''
static __device__ unsigned long long* g_guard_buf = nullptr;
__device__ __forceinline__ bool guard_bad(const void* p, int prim) {
    const unsigned long long u = (unsigned long long)p;
    const bool bad = u >= (1ull << 47) || u < 65536ull;
    if (bad && g_guard_buf) {
        __hip_atomic_fetch_add(g_guard_buf, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(g_guard_buf + 1 + 64 * prim + (threadIdx.x >> 6), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return __builtin_amdgcn_ballot_w64(bad) != 0;      // wave-uniform: the asm stays in uniform control flow
}
'''
PATCHES = [
    ("""__device__ __forceinline__ void glds16(const void* src, void* dst) {
    const unsigned off""", """__device__ __forceinline__ void glds16(const void* src, void* dst) {
    if (guard_bad(src, 0)) return;
    const unsigned off""", 1),
    ("""__device__ __forceinline__ void glds16_at(const void* src, void* base, int byte_off) {
    const unsigned off""", """__device__ __forceinline__ void glds16_at(const void* src, void* base, int byte_off) {
    if (guard_bad(src, 1)) return;
    const unsigned off""", 1),
    ("""__device__ __forceinline__ void glds4(const void* src, void* dst) {
    const unsigned off""", """__device__ __forceinline__ void glds4(const void* src, void* dst) {
    if (guard_bad(src, 2)) return;
    const unsigned off""", 1),
    ("""__device__ __forceinline__ void st_nt(float* p, const float4& v) {
    const v4f x""", """__device__ __forceinline__ void st_nt(float* p, const float4& v) {
    if (guard_bad(p, 3)) return;
    const v4f x""", 1),
    ("""__device__ __forceinline__ void st_tile(float* p, const float4& v) {
    const v4f x""", """__device__ __forceinline__ void st_tile(float* p, const float4& v) {
    if (guard_bad(p, 4)) return;
    const v4f x""", 1),
    ("void launch_stream(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen, bool half) {",
     """extern "C" int psgla_guard_set(void* p) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_guard_buf), &p, sizeof(p)); }
void launch_stream(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen, bool half) {""", 1),
    ("__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }",
     GUARD + """__device__ __forceinline__ float4 ld4(const float* p) {
    if (guard_bad(p, 5)) return make_float4(0.f, 0.f, 0.f, 0.f);
    return *reinterpret_cast<const float4*>(p);
}""", 1),
    ("            fM[r] = *reinterpret_cast<const uint32_t*>(a.mask + (size_t)b * a.m_cs + (size_t)gi[r] * L + gj0);",
     "            fM[r] = guard_bad(a.mask + (size_t)b * a.m_cs + (size_t)gi[r] * L + gj0, 6) ? 0u : *reinterpret_cast<const uint32_t*>(a.mask + (size_t)b * a.m_cs + (size_t)gi[r] * L + gj0);", 1),
    ("bool launch_tile(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen) {",
     """extern "C" int psgla_guard_set_tile(void* p) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_guard_buf), &p, sizeof(p)); }
bool launch_tile(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen) {""", 1),
    ("""    const long long step = launch_step(a);
    const bool fresh = launch_fresh(a);
    // the previous step's pending early-stop redo (rare): all workgroups in parallel, then one grid barrier;""",
     """    const long long step = launch_step(a);
    const bool fresh = launch_fresh(a);
    if ((step < 0 || step >= (1ll << 31)) && g_guard_buf && threadIdx.x == 0)
        __hip_atomic_store(g_guard_buf + 400, (unsigned long long)step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the previous step's pending early-stop redo (rare): all workgroups in parallel, then one grid barrier;""", 1),
]
