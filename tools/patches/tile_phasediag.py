# Diagnostic (never in the product): per-phase timeline of tv_tile_kernel.  Wave 0 of every workgroup stamps the
# 100 MHz real-time counter at 7 points of the main pass into a buffer set by psgla_tilediag_set_buffer(), slot
# [step & 1][blockIdx.x][i] (u64, 4096 workgroups per slot): 0 kernel entry, 1 loads issued + noise computed,
# 2 loads landed + data term + first barrier, 3 the inner iterations done, 4 rel-err atomics + X side + u2 stores
# issued, 5 arrival (stores complete, counter added), 6 end of the step finalisation (the last workgroup only).
# tools/tile_phasediag.py reads it.
DEFS = r'''
__device__ unsigned long long* g_tdiag = nullptr;
extern "C" int psgla_tilediag_set_buffer(void* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_tdiag), &p, sizeof(p));
}
__device__ __forceinline__ void tdiag(long long step, int i) {
    unsigned long long* const p = g_tdiag;
    // wave 0 stores (every lane the same value): a wave-uniform branch keeps the kernel's uniformity analysis intact
    if (p && __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0)
        p[((size_t)(step & 1) * 4096 + blockIdx.x) * 8 + i] = __builtin_amdgcn_s_memrealtime();
}

template <int R, int NW>
struct TileShared {'''
PATCHES = [
    ("\ntemplate <int R, int NW>\nstruct TileShared {", DEFS, 1),
    ("    // ---- 3. data term Y = (X + c1 g) + c2 Z, TV start state", "    if (track) tdiag(step, 1);\n    // ---- 3. data term Y = (X + c1 g) + c2 Z, TV start state", 1),
    ("    __syncthreads();\n    // The previous mean / sq of the core rows", "    __syncthreads();\n    if (track) tdiag(step, 2);\n    // The previous mean / sq of the core rows", 1),
    ("    if (n_it > 0) iteration(n_it - 1, std::true_type{}, std::integral_constant<int, 2>{});\n",
     "    if (n_it > 0) iteration(n_it - 1, std::true_type{}, std::integral_constant<int, 2>{});\n    if (track) tdiag(step, 3);\n", 1),
    ("            if (lo ? corelane_o : corelane) st_tile(lo ? pb : pa, v2);\n        }\n    }\n",
     "            if (lo ? corelane_o : corelane) st_tile(lo ? pb : pa, v2);\n        }\n    }\n    if (track) tdiag(step, 4);\n", 1),
    ("    const int P = a.B * a.C;\n    const int T = a.nbands", "    tdiag(step, 0);\n    const int P = a.B * a.C;\n    const int T = a.nbands", 1),
    ("            wait_vm0();\n            __syncthreads();\n        };", "            wait_vm0();\n            __syncthreads();\n            tdiag(step, 5);\n        };", 1),
    ("    if (threadIdx.x == 0) {\n        // both counts out", "    tdiag(step, 6);\n    if (threadIdx.x == 0) {\n        // both counts out", 1),
]
