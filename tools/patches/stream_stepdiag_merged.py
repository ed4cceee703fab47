# Step diagnostic of the merged stage layout (commit 8674423, PSGLA_STREAM_LAYOUT=2): the same stamps on that commit's sources
# (export them first: for f in api.hip tv_stream.hip tv_tile.hip psgla_common.hpp; do git show 8674423:psgla_for_posterior_sampling_amd/csrc/$f > /tmp/merged/$f; done)
# Diagnostic (never in the product): per-step barrier accounting of tv_stream_kernel with little perturbation.
# Every wave's lane 0 stamps its arrival (s_memtime) before each step barrier and its release after it; per-wave
# sums live in LDS.  Who arrived last: every arrival does an LDS max into the step's slot (parity-indexed; the
# times only grow, so a slot needs no reset), and at its next arrival each wave compares the closed step's max
# with its own previous arrival.  Workgroups 0..63 write [n, sum step length (wave 0), sum of the latest
# arrival - wave 0's release, per-wave work sums (16), per-wave last-arrival counts (16)] to the buffer set by
# psgla_stepdiag_set_buffer() (tools/stream_stepdiag.py).
DIAG = r'''
struct StepDiag {
    unsigned long long slot[2];
    unsigned long long prev_arr[16], rel[16], work[16], last[16];
    unsigned long long sum_step, sum_max, n;
    int cnt[16];
};
'''
FN = r'''
__device__ unsigned long long* g_sdiag = nullptr;
extern "C" int psgla_stepdiag_set_buffer(void* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_sdiag), &p, sizeof(p));
}
template <class SH>
__device__ __forceinline__ void diag_barrier(SH& sh) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    StepDiag& d = sh.sd;
    if (lane == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        const int c = d.cnt[w];
        if (c > 0) {
            const unsigned long long pm = d.slot[(c + 1) & 1];   // max arrival of step c - 1 (closed)
            if (c > 1 && pm == d.prev_arr[w]) d.last[w] += 1;
            d.work[w] += t1 - d.rel[w];
        }
        atomicMax(&d.slot[c & 1], t1);
        d.prev_arr[w] = t1;
        d.cnt[w] = c + 1;
    }
    lds_barrier();
    if (lane == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        if (w == 0) {
            const int c = d.cnt[0] - 1;
            if (c > 0) { d.sum_step += t0 - d.rel[0]; d.n += 1; }
        }
        d.rel[w] = t0;
    }
}
'''
import os as _os
_SRC = open("/tmp/merged/tv_stream.hip").read()
_N_BARRIER = _SRC.count("step_barrier();")
_SP = "HALF>" if "stream_pass<EXACT, ALPHA1, GEN, HALF>(a, sh, rm, a.n_tv" in _SRC else ">"
PATCHES = [
    ("template <bool A1>\nstruct StreamSharedT {\n", DIAG + "template <bool A1>\nstruct StreamSharedT {\n", 1),
    ("    float red[SP_MAXSEG][2][SP_MAXST][2];   // rel-err partial sums per (stream segment, half-wave, iteration)\n", "    float red[SP_MAXSEG][2][SP_MAXST][2];\n    StepDiag sd;\n", 1),
    ("\n\n// Row stream of a workgroup.", "\n" + FN + "\n// Row stream of a workgroup.", 1),
    ("step_barrier();", "diag_barrier(sh);", _N_BARRIER),
    ("        stream_pass<EXACT, ALPHA1, GEN, HALF, MRG>" + "(a, sh, rm, a.n_tv, true, step, fresh);\n",
     "        {\n"
     "            unsigned long long* z = reinterpret_cast<unsigned long long*>(&sh.sd);\n"
     "            for (int i = threadIdx.x; i < (int)(sizeof(StepDiag) / 8); i += blockDim.x) z[i] = 0;\n"
     "            __syncthreads();\n"
     "        }\n"
     "        stream_pass<EXACT, ALPHA1, GEN, HALF, MRG>" + "(a, sh, rm, a.n_tv, true, step, fresh);\n"
     "        __syncthreads();\n"
     "        if (g_sdiag && blockIdx.x < 64 && threadIdx.x == 0) {\n"
     "            unsigned long long* o = g_sdiag + (size_t)blockIdx.x * 64;\n"
     "            o[0] = sh.sd.n; o[1] = sh.sd.sum_step; o[2] = 0; o[3] = 0;\n"
     "            for (int i = 0; i < 16; ++i) { o[4 + i] = sh.sd.work[i]; o[20 + i] = sh.sd.last[i]; }\n"
     "        }\n", 1),
]

SOURCE_OVERRIDE = {f: "/tmp/merged/" + f for f in ("api.hip", "tv_stream.hip", "tv_tile.hip", "psgla_common.hpp")}
