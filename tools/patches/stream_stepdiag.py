# Diagnostic (never in the product): per-step barrier accounting of tv_stream_kernel.  Every wave stamps its
# arrival (s_memtime) into LDS before each step barrier; after the barrier, lane 0 of wave 15 (a back wave)
# reads the 16 arrival times of the step just closed and accumulates, per workgroup: the step length, the
# release latency after the last arrival, the latest arrival, which wave arrived last (histogram), and each
# wave's work (arrival - previous release of wave 15).  Workgroups 0..63 write their sums to the buffer set by
# psgla_stepdiag_set_buffer() (tools/stream_stepdiag.py).
DIAG = r'''
struct StepDiag {
    unsigned long long arr[2][16];
    unsigned long long prev_rel, sum_step, sum_gap, sum_max, n;
    unsigned long long work[16];
    unsigned long long last[16];
    int cnt[16];
};
'''
FN = r'''
__device__ unsigned long long* g_sdiag = nullptr;
extern "C" int psgla_stepdiag_set_buffer(void* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_sdiag), &p, sizeof(p));
}
__device__ __forceinline__ void diag_barrier(StreamShared& sh) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    StepDiag& d = sh.sd;
    const int c = d.cnt[w];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) { d.arr[c & 1][w] = t1; d.cnt[w] = c + 1; }
    lds_barrier();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (w == 15 && lane == 0) {
        unsigned long long mx = 0; int am = 0;
        for (int i = 0; i < 16; ++i) { const unsigned long long v = d.arr[c & 1][i]; if (v > mx) { mx = v; am = i; } }
        if (c > 0) {
            d.sum_step += t0 - d.prev_rel;
            d.sum_gap += t0 - mx;
            d.sum_max += mx - d.prev_rel;
            for (int i = 0; i < 16; ++i) d.work[i] += d.arr[c & 1][i] - d.prev_rel;
            d.last[am] += 1;
            d.n += 1;
        }
        d.prev_rel = t0;
    }
}
'''
PATCHES = [
    ("struct StreamShared {\n", DIAG + "struct StreamShared {\n", 1),
    ("    float red[SP_MAXSEG][SP_MAXST][2];\n};\n", "    float red[SP_MAXSEG][SP_MAXST][2];\n    StepDiag sd;\n};\n" + FN, 1),
    ("step_barrier();", "diag_barrier(sh);", 10),
    ("        stream_pass<EXACT, ALPHA1, GEN>(a, sh, rm, a.n_tv, true, step, fresh);\n",
     "        {\n"
     "            unsigned long long* z = reinterpret_cast<unsigned long long*>(&sh.sd);\n"
     "            for (int i = threadIdx.x; i < (int)(sizeof(StepDiag) / 8); i += blockDim.x) z[i] = 0;\n"
     "            __syncthreads();\n"
     "        }\n"
     "        stream_pass<EXACT, ALPHA1, GEN>(a, sh, rm, a.n_tv, true, step, fresh);\n"
     "        if (g_sdiag && blockIdx.x < 64 && threadIdx.x == 15 * 64) {\n"
     "            unsigned long long* o = g_sdiag + (size_t)blockIdx.x * 64;\n"
     "            o[0] = sh.sd.n; o[1] = sh.sd.sum_step; o[2] = sh.sd.sum_gap; o[3] = sh.sd.sum_max;\n"
     "            for (int i = 0; i < 16; ++i) { o[4 + i] = sh.sd.work[i]; o[20 + i] = sh.sd.last[i]; }\n"
     "        }\n", 1),
]
