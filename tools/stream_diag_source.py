"""Diagnostic variant of csrc/psgla_kernels.hip (never built into the product library): per-wave cycle
accounting of the row-stream kernel (tv_stream_kernel): work / wait per step, and the front waves' work
per pipeline phase.  Exports psgla_diag_set_buffer(device_ptr) for a caller-allocated
[workgroups][16][8] u64 buffer.  Usage:
    python3 tools/stream_diag_source.py /tmp/diag/psgla_diag.hip   (then hipcc it like build.py does;
    tools/stream_diag.py loads the result)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s = open(os.path.join(REPO, "psgla_for_posterior_sampling_amd", "csrc", "psgla_kernels.hip")).read()


def rep(old, new, count=1):
    global s
    if s.count(old) != count:
        raise SystemExit(f"pattern count {s.count(old)} != {count}: {old[:80]!r}")
    s = s.replace(old, new)


rep("""    int fin_inline;                 // stream kernel: 1 = the last workgroup finalises the step
""", """    int fin_inline;                 // stream kernel: 1 = the last workgroup finalises the step
    unsigned long long* diag;
""")
rep("""struct StepInfo {""", """struct Diag { unsigned long long t0 = 0, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; };
__device__ __forceinline__ unsigned long long dnow() {
    unsigned long long t;
    asm volatile("s_memtime %0\\n\\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    return t;
}
__device__ __forceinline__ void dbar1(Diag& d, int slot) {
    const unsigned long long t1 = dnow();
    d.acc[0] += t1 - d.t0;
    if (slot >= 0) d.acc[slot] += t1 - d.t0;
    lds_barrier();
    d.t0 = dnow();
    d.acc[1] += d.t0 - t1;
}
struct StepInfo {""")
# stage_loop signature and barriers
rep("""                                           int nsteps, int Qk, int lane, int lastk, int nreal, bool core) {""",
    """                                           int nsteps, int Qk, int lane, int lastk, int nreal, bool core, Diag& dg) {""")
i = s.index("__device__ __forceinline__ void stage_loop(")
j = s.index("// One pass of the row-streaming pipeline")
seg = s[i:j].replace("step_barrier();", "dbar1(dg, -1);")
s = s[:i] + seg + s[j:]
i = s.index("__device__ __forceinline__ void stream_pass(")
j = s.index("__global__ void __launch_bounds__(TV_THREADS) tv_stream_kernel(")
seg = s[i:j]
seg = seg.replace("""    const int lane = threadIdx.x & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (scalar branches)
""", """    const int lane = threadIdx.x & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (scalar branches)
    Diag dg;
    dg.t0 = dnow();
""", 1)
seg = seg.replace("lane, lastk, nreal, core);", "lane, lastk, nreal, core, dg);")
# front loop barrier (the one right after the front's if-block): first occurrence after 'FRONT ===='
k0 = seg.index("// ======================= FRONT =======================")
k1 = seg.index("step_barrier();", k0)
seg = seg[:k1] + "dbar1(dg, 2 + p);" + seg[k1 + len("step_barrier();"):]
seg = seg.replace("step_barrier();", "dbar1(dg, -1);")
# write-out before the end of stream_pass: after the back branch closes
k = seg.rindex("    // rel_err partial sums of this stream -> global")
seg = seg[:k] + """    if (a.diag && track && lane == 0)
        for (int q = 0; q < 8; ++q) a.diag[((size_t)blockIdx.x * 16 + w) * 8 + q] = dg.acc[q];
""" + seg[k:]
s = s[:i] + seg + s[j:]
rep("""    a.advance_step = d->advance_step;
""", """    a.advance_step = d->advance_step;
    a.diag = g_diag;
""")
rep("""static thread_local char g_err[512] = "";""", """static thread_local char g_err[512] = "";
static unsigned long long* g_diag = nullptr;      // diagnostic build: caller-allocated device buffer
extern "C" int psgla_diag_set_buffer(void* p) { g_diag = (unsigned long long*)p; return 0; }""")
open(sys.argv[1], "w").write(s)
