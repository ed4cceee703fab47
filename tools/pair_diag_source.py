"""Diagnostic variant of csrc/psgla_kernels.hip (never built into the product library): per-wave cycle
accounting of the row-pair kernel's phases.  Writes a patched copy of the source to argv[1]; the copy
exports psgla_diag_set_buffer(device_ptr) -- a caller-allocated [workgroups][16][12] u64 buffer that
receives, per wave, the shader cycles spent working / waiting in the W and C phases of the main pass
(slots 0-3) and, for waves 0-3, the work per front phase (4-7: C-phase, 8-11: W-phase by phs); for the
stage waves slots 4-5 split W / C work by whether the wave had noise duty that step.
    python3 tools/pair_diag_source.py /tmp/diag/psgla_diag.hip
    hipcc ... -shared -I include -I psgla_for_posterior_sampling_amd/csrc -o exp_libs/lib_diag.so /tmp/diag/psgla_diag.hip
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(os.path.join(REPO, "psgla_for_posterior_sampling_amd", "csrc", "psgla_kernels.hip")).read()


def rep(old, new, count=1):
    global s
    if s.count(old) != count:
        raise SystemExit(f"pattern count {s.count(old)} != {count}: {old[:80]!r}")
    s = s.replace(old, new)


rep("""    int pair;                       // stream kernel: 1 = the row-pair pipeline (tv_pair_kernel)
""", """    int pair;                       // stream kernel: 1 = the row-pair pipeline (tv_pair_kernel)
    unsigned long long* diag;
""")
rep("""// stream row q starts a segment (the stream's first row, or a plane start inside a split range)""",
    """struct Diag { unsigned long long t0 = 0, acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; };
__device__ __forceinline__ unsigned long long dnow() {
    unsigned long long t;
    asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    return t;
}
__device__ __forceinline__ void dbar(Diag& d, int ph, int slot = -1) {
    const unsigned long long t1 = dnow();
    d.acc[2 * ph] += t1 - d.t0;
    if (slot >= 0) d.acc[slot] += t1 - d.t0;
    lds_barrier();
    d.t0 = dnow();
    d.acc[2 * ph + 1] += d.t0 - t1;
}
// stream row q starts a segment (the stream's first row, or a plane start inside a split range)""")
rep("""                                           int T1, int lane, int lastk, bool core, long long stepi) {""",
    """                                           int T1, int lane, int lastk, bool core, long long stepi, Diag& dg) {""")
rep("""        noise(t, std::integral_constant<int, 0>());
        lds_barrier();""", """        noise(t, std::integral_constant<int, 0>());
        dbar(dg, 0);""")
rep("""        noise(t, std::integral_constant<int, 1>());
        lds_barrier();""", """        noise(t, std::integral_constant<int, 1>());
        dbar(dg, 1);""")
rep("""    const bool trk = track && role == 1 && (k_st - 1) >= 2 && (k_st - 1) <= n - 2;
    // (plane, plane row)""", """    const bool trk = track && role == 1 && (k_st - 1) >= 2 && (k_st - 1) <= n - 2;
    Diag dg;
    dg.t0 = dnow();
    // (plane, plane row)""")
# front: W barrier then C barrier inside its loop
i = s.index("        // ---------------- FRONT: pairs p = f, f + 4, ... ----------------")
j = s.index("    } else if (role == 1) {", i)
seg = s[i:j]
assert seg.count("            lds_barrier();\n") == 2
seg = seg.replace("            lds_barrier();\n", "            dbar(dg, 0, 8 + phs);\n", 1).replace("            lds_barrier();\n", "            dbar(dg, 1, 4 + phs);\n", 1)
s = s[:i] + seg + s[j:]
rep("""lane, lastk, lane_ok, step);
        else pair_stage<EXACT, false>(a, sh, rm, k_st, T0, T1, lane, lastk, lane_ok, step);
    } else if (role == 3) {
        for (int t = T0; t < T1; ++t) { lds_barrier(); lds_barrier(); }""", """lane, lastk, lane_ok, step, dg);
        else pair_stage<EXACT, false>(a, sh, rm, k_st, T0, T1, lane, lastk, lane_ok, step, dg);
    } else if (role == 3) {
        for (int t = T0; t < T1; ++t) { dbar(dg, 0); dbar(dg, 1); }""")
i = s.index("        // ---------------- BACK: steps t = bw (mod 2)")
j = s.index("template <bool EXACT>\n__global__ void __launch_bounds__(TV_THREADS) tv_pair_kernel", i)
seg = s[i:j]
assert seg.count("            lds_barrier();\n") == 2, seg.count("            lds_barrier();\n")
seg = seg.replace("            lds_barrier();\n", "            dbar(dg, 0, mine ? 8 : 9);\n", 1).replace("            lds_barrier();\n", "            dbar(dg, 1, mine ? 4 : 5);\n", 1)
# write-out at the very end of pair_pass (the back branch is the last one)
k = seg.rindex("    }\n}\n")
seg = seg[:k] + """    }
    if (a.diag && track && lane == 0)
        for (int q = 0; q < 12; ++q) a.diag[((size_t)blockIdx.x * 16 + w) * 12 + q] = dg.acc[q];
}
""" + seg[k + len("    }\n}\n"):]
s = s[:i] + seg + s[j:]
rep("""    a.advance_step = d->advance_step;
""", """    a.advance_step = d->advance_step;
    a.diag = g_diag;
""")
rep("""static thread_local char g_err[512] = "";""", """static thread_local char g_err[512] = "";
static unsigned long long* g_diag = nullptr;      // diagnostic build: caller-allocated device buffer
extern "C" int psgla_diag_set_buffer(void* p) { g_diag = (unsigned long long*)p; return 0; }""")
open(sys.argv[1], "w").write(s)
