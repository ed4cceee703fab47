// Memory-side probe of the row-stream pipeline's access pattern (diagnostic, never part of the product
// library; built by tools/mem_probe.sh into exp_libs/).  The stream kernel's HBM traffic WITHOUT its TV
// arithmetic: 256 row ranges (one 16-wave workgroup per CU), n_tv halo rows at each range end, the four
// front waves LDS-DMA a row's X, u2, y, mask, mean, sq four steps ahead (one front wave per row, as the
// stream kernel), the two back waves store X, u2, mean, sq of the row `depth` steps behind, one workgroup
// barrier per step.  Variants: 0 = that skeleton; 1 = front loads to VGPRs + ds_write (no LDS-DMA);
// 2 = no barrier (front / back free-running: the pattern's issue capacity); 3 = a plain grid-stride
// kernel moving the same bytes (the copy roofline of the same arrays).
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int WAVE = 64;
constexpr int NSLOT = 16;

struct ProbeArgs {
    const float* x; const float* u2; const float* y; const uint8_t* mask; const float* mean; const float* sq;
    float* xo; float* u2o; float* meano; float* sqo;
    int P, H, W;       // planes, rows, columns (W == 256)
    int nwg, halo, lead, depth, order;
};

struct ProbeShared {
    float4 st[NSLOT][6][WAVE];     // 96 KB
    uint32_t mk[NSLOT][WAVE];
};

typedef __attribute__((address_space(3))) void* lptr_t;
__device__ __forceinline__ void glds16(const void* src, void* dst) {
    const unsigned off = (unsigned)(size_t)(lptr_t)dst;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" :: "v"(src), "s"(off) : "memory", "m0");
}
__device__ __forceinline__ void glds4(const void* src, void* dst) {
    const unsigned off = (unsigned)(size_t)(lptr_t)dst;
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" :: "v"(src), "s"(off) : "memory", "m0");
}
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_nt(float* p, const float4& v) {
    const v4f x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 1" :: "v"(p), "v"(x) : "memory");
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int V>
__global__ void __launch_bounds__(1024) probe_kernel(const ProbeArgs a) {
    __shared__ ProbeShared sh;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long T = (long long)a.P * a.H;
    int b = blockIdx.x;
    if (a.order == 1) b = (b & 7) * (a.nwg / 8) + (b >> 3);     // XCD-contiguous ranges
    const long long c0 = T * b / a.nwg, c1 = T * (b + 1) / a.nwg;
    const long long l0 = c0 - a.halo < 0 ? 0 : c0 - a.halo;
    const long long l1 = c1 + a.halo > T ? T : c1 + a.halo;
    const int nload = (int)(l1 - l0);
    const int nsteps = nload + a.depth;
    const int col = 4 * lane;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 rX, rU0, rU1, rY, rM, rS;
    uint32_t rMk = 0;
    if (V == 2 && w >= 4 && w < 14) return;
    for (int s = 0; s < nsteps; ++s) {
        if (w < 4 && (s & 3) == w) {
            wait_vm0();
            const int ip = s - 4 + a.lead;          // the row this wave loaded 4 steps ago
            if (V == 1 && s >= 4 && ip < nload) {
                const int sl = ip & (NSLOT - 1);
                sh.st[sl][0][lane] = rX; sh.st[sl][1][lane] = rU0; sh.st[sl][2][lane] = rU1;
                sh.st[sl][3][lane] = rY; sh.st[sl][4][lane] = rM; sh.st[sl][5][lane] = rS;
                sh.mk[sl][lane] = rMk;
            }
            const int i = s + a.lead;
            if (i < nload) {
                const long long g = l0 + i;
                const bool core = g >= c0 && g < c1;
                const size_t off = (size_t)g * a.W + col;
                const size_t yoff = off;                                     // y per chain (bench.py)
                const size_t moff = (size_t)(g % a.H) * a.W + col;
                const int sl = i & (NSLOT - 1);
                if (V == 1) {
                    rX = *reinterpret_cast<const float4*>(a.x + off);
                    rU0 = *reinterpret_cast<const float4*>(a.u2 + 2 * off);
                    rU1 = *reinterpret_cast<const float4*>(a.u2 + 2 * off + 4);
                    rY = *reinterpret_cast<const float4*>(a.y + yoff);
                    rMk = *reinterpret_cast<const uint32_t*>(a.mask + moff);
                    if (core) {
                        rM = *reinterpret_cast<const float4*>(a.mean + off);
                        rS = *reinterpret_cast<const float4*>(a.sq + off);
                    }
                } else {
                    glds16(a.x + off, &sh.st[sl][0][0]);
                    glds16(a.u2 + 2 * off, &sh.st[sl][1][0]);
                    glds16(a.u2 + 2 * off + 4, &sh.st[sl][2][0]);
                    glds16(a.y + yoff, &sh.st[sl][3][0]);
                    glds4(a.mask + moff, &sh.mk[sl][0]);
                    if (core) {
                        glds16(a.mean + off, &sh.st[sl][4][0]);
                        glds16(a.sq + off, &sh.st[sl][5][0]);
                    }
                }
            }
        } else if (w >= 14) {
            const int i = s - a.depth;
            if (i >= 0 && i < nload) {
                const long long g = l0 + i;
                const int sl = (s + 1) & (NSLOT - 1);
                const float4 v = sh.st[sl][w - 14][lane];
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
                if (g >= c0 && g < c1) {
                    const size_t off = (size_t)g * a.W + col;
                    if (w == 14) {
                        st_nt(a.xo + off, acc);
                        st_nt(a.u2o + 2 * off, acc);
                        st_nt(a.u2o + 2 * off + 4, acc);
                    } else {
                        st_nt(a.meano + off, acc);
                        st_nt(a.sqo + off, acc);
                    }
                }
            }
        }
        if (V != 2) bar();
    }
    wait_vm0();
}


// ---- variant 4 / 5: the memory skeleton plus synthetic per-role work of the stream kernel's size
// (stage wave: ring k-1 + Y reads, ~140 VALU, ring k writes; front: ~50 VALU per phase + the data-term
// phase's staging reads and ring-0 / Y writes; back: ring n reads + ~30 VALU).  DMAW 0: the row's front
// wave issues its DMAs (as the stream kernel); DMAW 1: stage wave 1 issues every row's DMAs and waits
// for them one step before the row is consumed.
constexpr int WSLOT = 8;
struct WorkShared {
    float4 st[WSLOT][6][WAVE];
    uint32_t mk[WSLOT][WAVE];
    float4 ring[11][2][3][WAVE];
    float4 yr[16][WAVE];
};

template <int NF>
__device__ __forceinline__ float4 burn(float4 v, float c) {
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        v.x = __builtin_fmaf(v.x, c, 0.5f);
        v.y = __builtin_fmaf(v.y, c, 0.25f);
        v.z = __builtin_fmaf(v.z, c, 0.125f);
        v.w = __builtin_fmaf(v.w, c, 0.0625f);
    }
    return v;
}

template <int DMAW>
__global__ void __launch_bounds__(1024) probe_work_kernel(const ProbeArgs a) {
    __shared__ WorkShared sh;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long T = (long long)a.P * a.H;
    const int b = blockIdx.x;
    const long long c0 = T * b / a.nwg, c1 = T * (b + 1) / a.nwg;
    const long long l0 = c0 - a.halo < 0 ? 0 : c0 - a.halo;
    const long long l1 = c1 + a.halo > T ? T : c1 + a.halo;
    const int nload = (int)(l1 - l0);
    const int nsteps = nload + a.depth;
    const int col = 4 * lane;
    const float cf = 0.999f;
    const bool nodma = (a.order & 2) != 0, nost = (a.order & 4) != 0;
    const bool nonoise = (a.order & 8) != 0, halfstage = (a.order & 16) != 0;
    auto issue_part = [&](int i, int part) {
        if (nodma) return;
        const long long g = l0 + i;
        const bool core = g >= c0 && g < c1;
        const size_t off = (size_t)g * a.W + col;
        const size_t moff = (size_t)(g % a.H) * a.W + col;
        const int sl = i & (WSLOT - 1);
        switch (part) {
            case 0: glds16(a.x + off, &sh.st[sl][0][0]); break;
            case 1: glds16(a.u2 + 2 * off, &sh.st[sl][1][0]); break;
            case 2: glds16(a.u2 + 2 * off + 4, &sh.st[sl][2][0]); break;
            case 3: glds16(a.y + off, &sh.st[sl][3][0]); break;
            case 4: glds4(a.mask + moff, &sh.mk[sl][0]); break;
            case 5: if (core) glds16(a.mean + off, &sh.st[sl][4][0]); break;
            default: if (core) glds16(a.sq + off, &sh.st[sl][5][0]); break;
        }
    };
    auto issue = [&](int i) {
        if (nodma) return;
        const long long g = l0 + i;
        const bool core = g >= c0 && g < c1;
        const size_t off = (size_t)g * a.W + col;
        const size_t moff = (size_t)(g % a.H) * a.W + col;
        const int sl = i & (WSLOT - 1);
        glds16(a.x + off, &sh.st[sl][0][0]);
        glds16(a.u2 + 2 * off, &sh.st[sl][1][0]);
        glds16(a.u2 + 2 * off + 4, &sh.st[sl][2][0]);
        glds16(a.y + off, &sh.st[sl][3][0]);
        glds4(a.mask + moff, &sh.mk[sl][0]);
        if (core) {
            glds16(a.mean + off, &sh.st[sl][4][0]);
            glds16(a.sq + off, &sh.st[sl][5][0]);
        }
    };
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (w < 4) {
        __builtin_amdgcn_s_setprio(0);
        for (int s = 0; s < nsteps; ++s) {
            const int p = (s + 4 - w) & 3;        // phase of this wave's current row q = s - p
            const int q = s - p;
            if (q >= 0 && q < nload) {
                if (p < 3) {
                    if (!nonoise) acc = burn<12>(acc, cf);
                } else {
                    if (DMAW == 0) wait_vm0();
                    const int sl = q & (WSLOT - 1);
                    float4 v = sh.st[sl][0][lane];
                    const float4 u0 = sh.st[sl][1][lane], u1 = sh.st[sl][2][lane], yy = sh.st[sl][3][lane];
                    v.x += u0.x + u1.x + yy.x + (float)(sh.mk[sl][lane] & 1u);
                    v = burn<8>(v, cf);
                    sh.ring[0][q & 1][0][lane] = v;
                    sh.ring[0][q & 1][1][lane] = u0;
                    sh.ring[0][q & 1][2][lane] = u1;
                    sh.yr[q & 15][lane] = acc;
                }
                if (DMAW == 0 && p == 3 && q + 4 + a.lead - 4 < nload) issue(q + a.lead);
            }
            bar();
        }
    } else if (w < 14) {
        const int k = w - 3;                          // stage 1..10: row q = s - 4 - 3 (k - 1) ... one per step
        __builtin_amdgcn_s_setprio(1);
        for (int s = 0; s < nsteps; ++s) {
            if (DMAW == 1 && k == 1) {
                const int i = s + a.lead;
                if (i < nload) issue(i);
                // rows consumed next step (q = s + 1 - 3) landed: the rows issued after it may fly
                asm volatile("s_waitcnt vmcnt(35)" ::: "memory");
            }
            if (DMAW == 2 && k <= 7) {
                const int i = s + a.lead;
                if (i < nload) issue_part(i, k - 1);
                asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
            }
            const int q = s - 4 - 3 * (k - 1);
            if (q >= 0 && q < nload) {
                float4 x = sh.ring[k - 1][q & 1][0][lane];
                float4 u0 = sh.ring[k - 1][q & 1][1][lane];
                float4 u1 = sh.ring[k - 1][q & 1][2][lane];
                const float4 yy = sh.yr[q & 15][lane];
                x.x += yy.x; u0.y += yy.y;
                if (halfstage) {
                    x = burn<6>(x, cf);
                    u0 = burn<6>(u0, cf);
                    u1 = burn<6>(u1, cf);
                } else {
                    x = burn<12>(x, cf);
                    u0 = burn<12>(u0, cf);
                    u1 = burn<11>(u1, cf);
                }
                sh.ring[k][q & 1][0][lane] = x;
                sh.ring[k][q & 1][1][lane] = u0;
                sh.ring[k][q & 1][2][lane] = u1;
            }
            bar();
        }
    } else {
        __builtin_amdgcn_s_setprio(3);
        for (int s = 0; s < nsteps; ++s) {
            const int i = s - a.depth;
            if (i >= 0 && i < nload && (i & 1) == (w - 14)) {
                const long long g = l0 + i;
                float4 x = sh.ring[10][i & 1][0][lane];
                const float4 u0 = sh.ring[10][i & 1][1][lane], u1 = sh.ring[10][i & 1][2][lane];
                x = burn<8>(x, cf);
                if (g >= c0 && g < c1 && !nost) {
                    const size_t off = (size_t)g * a.W + col;
                    st_nt(a.xo + off, x);
                    st_nt(a.u2o + 2 * off, u0);
                    st_nt(a.u2o + 2 * off + 4, u1);
                    st_nt(a.meano + off, x);
                    st_nt(a.sqo + off, u0);
                }
            }
            bar();
        }
    }
    wait_vm0();
}

// the same bytes by a plain grid-stride copy: per row, read X, u2, y, mask, mean, sq, write X, u2, mean, sq
__global__ void __launch_bounds__(256) probe_copy_kernel(const ProbeArgs a) {
    const long long T = (long long)a.P * a.H;
    const long long n = T * (a.W / 4);
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
        const long long g = q / (a.W / 4);
        const int col = 4 * (int)(q % (a.W / 4));
        const size_t off = (size_t)g * a.W + col;
        const size_t yoff = off;
        const size_t moff = (size_t)(g % a.H) * a.W + col;
        const float4 X = *reinterpret_cast<const float4*>(a.x + off);
        const float4 U0 = *reinterpret_cast<const float4*>(a.u2 + 2 * off);
        const float4 U1 = *reinterpret_cast<const float4*>(a.u2 + 2 * off + 4);
        const float4 Y = *reinterpret_cast<const float4*>(a.y + yoff);
        const uint32_t mk = *reinterpret_cast<const uint32_t*>(a.mask + moff);
        const float4 M = *reinterpret_cast<const float4*>(a.mean + off);
        const float4 S = *reinterpret_cast<const float4*>(a.sq + off);
        const float f = (float)(mk & 1u);
        st_nt(a.xo + off, make_float4(X.x + Y.x * f, X.y + Y.y, X.z + Y.z, X.w + Y.w));
        st_nt(a.u2o + 2 * off, U0);
        st_nt(a.u2o + 2 * off + 4, U1);
        st_nt(a.meano + off, M);
        st_nt(a.sqo + off, S);
    }
}

extern "C" int probe_launch(const ProbeArgs* a, int variant, int copy_grid, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    switch (variant) {
        case 0: hipLaunchKernelGGL(probe_kernel<0>, dim3(a->nwg), dim3(1024), 0, st, *a); break;
        case 1: hipLaunchKernelGGL(probe_kernel<1>, dim3(a->nwg), dim3(1024), 0, st, *a); break;
        case 2: hipLaunchKernelGGL(probe_kernel<2>, dim3(a->nwg), dim3(1024), 0, st, *a); break;
        case 3: hipLaunchKernelGGL(probe_copy_kernel, dim3(copy_grid), dim3(256), 0, st, *a); break;
        case 4: hipLaunchKernelGGL(probe_work_kernel<0>, dim3(a->nwg), dim3(1024), 0, st, *a); break;
        case 5: hipLaunchKernelGGL(probe_work_kernel<1>, dim3(a->nwg), dim3(1024), 0, st, *a); break;
        case 6: hipLaunchKernelGGL(probe_work_kernel<2>, dim3(a->nwg), dim3(1024), 0, st, *a); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
