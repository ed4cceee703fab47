// Shared device code of libpsgla_hip (MI355X, gfx950): the TV step's argument block, the LDS-DMA /
// store / wait primitives, the schedule helpers, and the host-side launch helpers every translation unit
// uses.  The kernels live in tv_stream.hip, tv_tile.hip, tv_band.hip, blur.hip and elementwise.hip; the C ABI
// (include/psgla_hip.h) in api.hip and next to the kernels it launches.  One translation unit per kernel
// family, so the library builds in parallel (build.py).
#pragma once
//
// libpsgla_hip: MI355X (gfx950, CDNA4) kernels for the PSGLA / PnP-ULA Langevin step.
//
// Hot path (reference /root/reference/restoration_algorithms.py):
//   psgla loop body   :231-271   Z ~ N(0,1); Y = X + (delta/lambd) g(X) + sqrt2 s Z;
//                                 X = (1-alpha) Y + alpha D(Y, s); block means of X, X^2
//   pnpula loop body  :103-144   X += delta (gp - (X - clip(X))/lambd + gd) + sqrt(2 delta) Z
//   g(X) (inpainting) sampling_images.py:295   -mask (x - y) / sigma2
//   D = TV prox       deepinv 0.2.1 TVDenoiser (sampling_images.py:138), warm-started
//
// Design: one fused kernel per Langevin step for PSGLA+TV.  A workgroup
// of 16 waves owns a band of up to 64 rows x 256 columns of one (chain, channel)
// plane; every lane owns 4 consecutive columns of 4 rows, so the whole TV state
// (x2, u2) and tau*Y of the tile live in registers for all inner iterations.  The
// inner iterations are temporally blocked: the band carries a halo of n_tv rows /
// columns (the stencil's dependency cone grows by one pixel per iteration), which is
// recomputed by neighbouring bands instead of being exchanged.  Horizontal
// neighbours are lane shuffles, vertical neighbours across waves go through two
// 16 KB LDS row buffers.  HBM traffic per element and step: read X, u2, y, mask,
// mean, sq; write X, u2, mean, sq (44.33 B with the 1-byte mask shared by 3
// channels); the Gaussian noise is generated in registers (Philox4x32-10).
//
// Floating-point: the library is compiled with -ffp-contract=off.  EXACT=true
// kernels evaluate the reference's expressions in the reference's order with IEEE
// division and square root and are bit-identical to the torch CPU checker
// (oracle/); EXACT=false replaces the four TV divisions and the sqrt by
// reciprocal/rsqrt forms and fmas (about 3x fewer VALU ops) and is checked against
// the same checker within the north-star tolerance.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cmath>
#include <stdint.h>
#include <type_traits>
#include <stdio.h>
#include <string.h>

#include "psgla_hip.h"
#include "noise.hpp"

// host side (api.hip): the library's last error message and the two ways of setting it
extern thread_local char g_err[512];
int fail(int code, const char* msg);
int launch_check(const char* what);

// x-extent of a (work items of one chain / plane, chains) grid: ~4 waves of workgroups over the CUs
static inline int grid_chain(long long per_chain, int chains) {
    long long g = (per_chain + 255) / 256;
    const long long cap = (4LL * 256 + chains - 1) / chains;   // total ~ 4 x 256 CUs x ... workgroups
    if (g > cap * 4) g = cap * 4;
    if (g < 1) g = 1;
    return (int)g;
}

static inline int grid_for(long long n, int threads) {
    long long g = (n + threads - 1) / threads;
    if (g > 256 * 16) g = 256 * 16;
    if (g < 1) g = 1;
    return (int)g;
}

namespace psgla {

constexpr int WAVE = 64;
constexpr int CPL = 4;            // columns per lane
constexpr int TV_R = 4;           // rows per wave
constexpr int TV_NW = 16;         // waves per workgroup
constexpr int TV_THREADS = TV_NW * WAVE;
constexpr int TV_ROWS = TV_NW * TV_R;      // 64 rows per band (with halo)
constexpr int TV_COLS = CPL * WAVE;        // 256 columns per segment (with halo)
constexpr int MAXIT = PSGLA_TV_MAX_FUSED_IT;
constexpr int MAXG = 1024;        // chains per launch (early-stop groups)
constexpr uint32_t TAG_LANGEVIN = 0;

// deepinv 0.2.1 TVDenoiser's step constants (tau = 0.01, rho = 1.99, sigma = 1 / tau / 8: fixed by
// /root/reference/sampling_images.py:138, which never passes others) in fp32, as the FAST kernels' compile-time
// operands.  Round 6 (tools/valu_probe2, profiles/r06q_valu_probe.txt): at 4 waves per SIMD a VALU instruction
// with an SGPR source costs 4.24-4.30 SIMD cycles per wave-instruction, one with a literal (v_fmamk_f32,
// VOP2 literal) 2.57 whatever the VGPR banks of the others, VGPR-only 2.17 / 2.57 (VOP2 / VOP3) unless two of three
// sources share a bank (4.24-4.39).  A fast request with other constants runs the exact kernels (api.hip:
// tv_fast_constants) -- the fast arithmetic, and so every fast result, is unchanged.
constexpr float TV_TAU = 0x1.47ae14p-7f;       // fp32(0.01)
constexpr float TV_OPT = 0x1.028f5cp+0f;       // fp32(1 + 0.01)
constexpr float TV_INV_OPT = 0x1.faee42p-1f;   // fp32(1 / (double)fp32(1.01)), TvArgs::inv_opt
constexpr float TV_SIG = 12.5f;                // fp32(1 / 0.01 / 8)
constexpr float TV_RHO = 0x1.fd70a4p+0f;       // fp32(1.99)

enum Front { FRONT_INPAINT = 0, FRONT_GIVEN = 1 };

struct TvArgs {
    int B, C, H, W;
    int ldw;                        // row pitch of every (.., H, W) buffer in elements (stream kernel; >= W)
    float* x[2];
    float* u2[2];
    float* x2[2];
    float* mean[2];
    float* sq[2];
    const float* yin;               // FRONT_GIVEN input
    const float* yobs;              // observation
    long long y_cs;
    const uint8_t* mask;
    long long m_cs;
    float c1, c2, sigma2, alpha;
    float inv_sigma2;               // fast kernels: 1/sigma2 (the data term multiplies)
    float tau, opt, inv_opt, sig_tv, rho, ths, tol;
    int n_tv;
    unsigned long long seed;
    int chain0;
    int pingpong;                   // 1: buffers indexed by step parity
    long long* d_step;
    long long step_offset;
    int fresh_host;
    int* fresh_dev;
    int per_chain_norm;
    int it0;                        // psgla_tv_prox chunks: global index of the first inner iteration
    int last_chunk;                 // 1: the call's last chunk (a stop at its last iteration changes nothing)
    int* stopped;                   // psgla_tv_prox chunks: [groups] stop count of the chunk (0: none)
    double* norms;
    int* arrive;
    int advance_step;
    // schedule
    int n_inter, nm;
    const float* coef;
    float* samples;
    long long samples_cap;
    float* blocks;
    float* blocks2;
    long long blocks_cap;
    // tiling
    int nbands, band_h, nsegs, seg_w, tiles, halo;
    int stream;                     // 1: main pass = row-streaming pipeline kernel
    int split_wgs;                  // stream kernel: > 0 = row-split mode over this many workgroups
    int st_nsegs, st_seg_w, st_halo;  // stream kernel column segmentation (W > 256)
    int st_half;                    // stream kernel: 1 = half windows (two 128-column segments per wave, one per
                                    // half-wave; 256 < W <= 324 at n_tv = 10: a third of the lanes fewer idle)
    int st_nvp;                     // stream kernel virtual planes: (plane, segment) items, or pairs of them (st_half)
    int fin_inline;                 // stream kernel: 1 = the last workgroup finalises the step
    int tile_r;                     // > 0: small-batch tile kernel with tile_r rows per wave (one tile per workgroup)
    int tile_nw;                    // tile kernel: waves per workgroup (16 or 8)
    int norm_copies;                // tile kernel: copies of norms its rel-err sums are spread over (>= 1)
    int* redo;                      // stream / tile kernel: parallel early-stop redo state (PsglaTvStep.redo) or null
    int par_redo;                   // 1: the redo runs in parallel in the next launch (grid resident at once)
    int redo_only;                  // 1: settle a pending redo only (launch_mask 4)
};

// The launch's step index and TV restart flag, wave-uniform by construction (readfirstlane: code that stores to
// global memory before using them must not make the compiler treat them as per-lane values)
__device__ __forceinline__ long long launch_step(const TvArgs& a) {
    const long long v = (a.d_step ? *a.d_step : 0LL) + a.step_offset;
    const int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xFFFFFFFFLL));
    const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ bool launch_fresh(const TvArgs& a) {
    return __builtin_amdgcn_readfirstlane(a.fresh_dev ? *a.fresh_dev : a.fresh_host) != 0;
}

// Grid-wide barrier of a launch whose workgroups are all resident (the parallel early-stop redo only): each
// workgroup's stores drained and released (agent scope), one arrival per workgroup on *cnt, a bounded poll, an
// agent acquire (MI355X_MICROARCH.md, valid hand-off form).  An expired guard is recorded in *guard for the host.
__device__ __forceinline__ void grid_sync(int* cnt, int* guard) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool done = false;
        for (int spin = 0; spin < (1 << 24) && !done; ++spin) {
            done = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (int)gridDim.x;
            if (!done) __builtin_amdgcn_s_sleep(2);
        }
        if (!done) __hip_atomic_store(guard, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// Inner iterations (chunk-local) whose rel_err deepinv tests: global index >= 2 ("it > 1"); in the call's
// last chunk not the last iteration (stopping there changes nothing)
__device__ __forceinline__ int trk_lo(const TvArgs& a) { return a.it0 >= 2 ? 0 : 2 - a.it0; }
__device__ __forceinline__ int trk_hi(const TvArgs& a) { return a.last_chunk ? a.n_tv - 2 : a.n_tv - 1; }

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float a, float b, float c, float d) {
    *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ float f4get(const float4& v, int k) {
    return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}

// Sum over the 64 lanes, returned in every lane.  DPP within each row of 16 lanes (xor 1, xor 2 by
// quad_perm, then row rotations by 4 and 8: every lane holds its row's sum), then the four row sums
// read out by v_readlane: pure VALU, no LDS round trips (a __shfl_xor tree is six dependent
// ds_bpermute's, ~0.5 us per tracked TV iteration on the tile kernel's critical path).
#define PSGLA_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), (ctrl), 0xF, 0xF, false))
__device__ __forceinline__ float wave_sum(float v) {
    v += PSGLA_DPP(v, 0xB1);      // quad_perm [1,0,3,2]: lane ^ 1
    v += PSGLA_DPP(v, 0x4E);      // quad_perm [2,3,0,1]: lane ^ 2
    v += PSGLA_DPP(v, 0x124);     // row_ror:4
    v += PSGLA_DPP(v, 0x128);     // row_ror:8
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}
// Sums over each 16-lane row, returned in every lane of the row (the first 4 steps of wave_sum).
// A kernel constant (an SGPR) copied once into a VGPR for 2-source VALU operands (4.24 -> 2.17 SIMD cycles per
// wave-instruction at 4 waves per SIMD, above); non-volatile asm, so it is CSE'd and hoisted out of loops
__device__ __forceinline__ float vconst(float s) {
    float v;
    asm("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
    return v;
}

// the TV dual's projection factor min(1, ths / |v|) = min(1, ths * rsq(s2)) as one multiply with the clamp
// modifier (fminf(fmaxf(x, 0), 1) folds to v_mul_f32_e64 ... clamp): identical for x >= 0 and +inf, and no v_min
// (4.24 SIMD cycles per wave-instruction at 4 waves per SIMD)
__device__ __forceinline__ float tv_proj_factor(float ths_v, float s2) {
    return fminf(fmaxf(ths_v * __builtin_amdgcn_rsqf(s2), 0.0f), 1.0f);
}

__device__ __forceinline__ float2 row_sum2(float a, float b) {
    a += PSGLA_DPP(a, 0xB1); b += PSGLA_DPP(b, 0xB1);      // quad_perm [1,0,3,2]
    a += PSGLA_DPP(a, 0x4E); b += PSGLA_DPP(b, 0x4E);      // quad_perm [2,3,0,1]
    a += PSGLA_DPP(a, 0x124); b += PSGLA_DPP(b, 0x124);    // row_ror:4
    a += PSGLA_DPP(a, 0x128); b += PSGLA_DPP(b, 0x128);    // row_ror:8
    return make_float2(a, b);
}
#undef PSGLA_DPP

// Block-mean accumulator + sample storage for one element (restoration_algorithms.py:240-271).
// idx = chain*E + e within the batch; BE = B*E (slot stride of samples/blocks).
__device__ __forceinline__ void accumulate_elem(const TvArgs& a, long long step, size_t idx, size_t BE,
                                                float X, const float* mean_in, const float* sq_in,
                                                float* mean_out, float* sq_out) {
    if (a.nm >= 0 && mean_out != nullptr) {
        const int per = a.nm + 1;
        const int im = (int)(step % per);
        const float ca = a.coef[2 * im], cb = a.coef[2 * im + 1];
        float m, q;
        if (im == 0) {
            m = cb * X;
            q = cb * (X * X);
        } else {
            m = ca * mean_in[idx] + cb * X;
            q = ca * sq_in[idx] + cb * (X * X);
        }
        if (im == a.nm) {
            const long long blk = step / per;
            if (blk < a.blocks_cap) {
                a.blocks[(size_t)blk * BE + idx] = m;
                a.blocks2[(size_t)blk * BE + idx] = q;
            }
        } else {
            mean_out[idx] = m;
            sq_out[idx] = q;
        }
    }
    if (a.n_inter > 0 && a.samples != nullptr && (step % a.n_inter) == 0) {
        const long long k = step / a.n_inter;
        if (k < a.samples_cap) a.samples[(size_t)k * BE + idx] = X;
    }
}


constexpr int SP_FRONT = 4;
constexpr int SP_BACK = 2;
constexpr int SP_MAXST = 10;
constexpr int SP_YRING = 32;
constexpr int SP_MAXSEG = 4;      // planes touched by one workgroup's row stream (split mode)
constexpr int SP_NOSEG = 1 << 30; // "no further segment start"

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
typedef float v4f_t __attribute__((ext_vector_type(4)));

// 16 B (4 B) per lane from global memory straight into LDS; lane i lands at dst + 16 i (4 i).
// Issued as inline asm: the compiler does not track these loads, so it cannot insert a
// conservative vmcnt(0) before unrelated LDS accesses -- the waves wait with counted
// s_waitcnt vmcnt(N) themselves (vector-memory operations retire in issue order).
__device__ __forceinline__ void glds16(const void* src, void* dst) {
    const unsigned off = (unsigned)(size_t)(lptr_t)dst;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(src), "s"(off) : "memory", "m0");
}
// glds16 at base + byte_off for a base whose LDS address folds to a constant (a __shared__ array) and a
// wave-uniform offset, forced into a scalar register: a call site the compiler cannot prove uniform (the tile
// kernel's second, early-stop redo, instance of its tile) otherwise leaves the m0 operand in a VGPR
__device__ __forceinline__ void glds16_at(const void* src, void* base, int byte_off) {
    const unsigned off = (unsigned)(size_t)(lptr_t)base + (unsigned)__builtin_amdgcn_readfirstlane(byte_off);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(src), "s"(off) : "memory", "m0");
}
__device__ __forceinline__ void glds4(const void* src, void* dst) {
    const unsigned off = (unsigned)(size_t)(lptr_t)dst;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
                 :: "v"(src), "s"(off) : "memory", "m0");
}
// Workgroup barrier that only drains LDS (lgkmcnt): LDS-DMA loads stay in flight across it
// (a __syncthreads() fence would wait vmcnt(0) while a global_load_lds is pending).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }
__device__ __forceinline__ void wait_vm0() { wait_vm<0>(); }
// vmcnt(n) for a wave-uniform n in [0, 23] (larger n waits for 23)
template <int N>
__device__ __forceinline__ void wait_vm_le(int n) {
    if constexpr (N >= 23) {
        wait_vm<23>();
    } else {
        if (n == N) wait_vm<N>();
        else wait_vm_le<N + 1>(n);
    }
}
__device__ __forceinline__ void wait_vm_n(int n) { wait_vm_le<0>(n); }
// 16-B streaming store (nt: the output rows are not re-read by this kernel).  Measured against
// plain, sc1 and sc0 sc1 stores on the bench step: nt is the fastest (the per-workgroup agent
// release before the arrival count still writes back whatever the XCD's L2 holds dirty).
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_nt(float* p, const float4& v) {
    const v4f x = {v.x, v.y, v.z, v.w};
    // s_nop: the compiler does not see this store, so it cannot pad the store-data hazard
    // (a VALU write of the data VGPRs right after a >8-byte store) -- the asm does
    asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
}

// Output store of the tile kernel: write-through (sc1) by default -- all its workgroups finish together
// and each then releases (writes back) its XCD's dirty L2 lines before the arrival count, which
// write-through stores leave clean (nt stores, as the stream kernel's, measured 17 % slower here).
__device__ __forceinline__ void st_tile(float* p, const float4& v) {
    const v4f x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
}

// end of a pipeline step: the workgroup barrier (LDS drained, LDS-DMA loads stay in flight)
__device__ __forceinline__ void step_barrier() { lds_barrier(); }

struct StepInfo {
    bool acc, first, blockend, liveout, sample;
    long long blk, sidx;
    float ca, cb;
};

__device__ __forceinline__ StepInfo step_info(const TvArgs& a, long long step, const float* mean_out) {
    StepInfo si;
    si.acc = a.nm >= 0 && mean_out != nullptr;
    const int per = a.nm + 1;
    const int im = si.acc ? (int)(step % per) : 0;
    si.first = im == 0;
    si.blk = si.acc ? step / per : 0;
    si.liveout = si.acc && im != a.nm;
    si.blockend = si.acc && im == a.nm && si.blk < a.blocks_cap;
    si.ca = si.acc ? a.coef[2 * im] : 0.f;
    si.cb = si.acc ? a.coef[2 * im + 1] : 0.f;
    si.sample = a.n_inter > 0 && a.samples != nullptr && (step % a.n_inter) == 0;
    si.sidx = si.sample ? step / a.n_inter : 0;
    si.sample = si.sample && si.sidx < a.samples_cap;
    return si;
}

// Core rows whose mean / sq rows a tile stages in LDS: all rows of the tile, at most 56 (112 KB; a 72-row tile
// of 8 waves x 9 rows has 52 core rows at n_tv = 10 -- tile_geometry keeps band_h within this)
constexpr int tile_mst_rows(int nw, int r) { return nw * r < 56 ? nw * r : 56; }

// kernel launchers (one translation unit each)
template <bool EXACT, int FRONT, bool ALPHA1> void launch_band_main(const TvArgs& a, dim3 grid, hipStream_t st);
template <bool EXACT, int FRONT, bool ALPHA1> void launch_band_finalise(const TvArgs& a, dim3 grid, hipStream_t st);
void launch_stream(const TvArgs& a, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen, bool half);
bool launch_tile(const TvArgs& a, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen);
// workgroups of the instance launch_stream / launch_tile would run that one CU holds at once (the runtime's occupancy
// query, cached per instance; 0 if unknown): the parallel early-stop redo's grid barrier needs the grid resident
int stream_blocks_per_cu(bool exact, bool alpha1, bool gen, bool half);
int tile_blocks_per_cu(const TvArgs& a, bool exact, bool alpha1, bool gen);

// cached hipOccupancyMaxActiveBlocksPerMultiprocessor of one kernel instance (slot: the instance's index)
static inline int occupancy_cached(int* cache, int slot, const void* kernel, int threads) {
    if (cache[slot] < 0) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, threads, 0) != hipSuccess) n = 0;
        cache[slot] = n;
    }
    return cache[slot];
}

}  // namespace psgla
