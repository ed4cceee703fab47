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
    int fin_inline;                 // stream kernel: 1 = the last workgroup finalises the step
    int tile_r;                     // > 0: small-batch tile kernel with tile_r rows per wave (one tile per workgroup)
    int tile_nw;                    // tile kernel: waves per workgroup (16 or 8)
    int norm_copies;                // tile kernel: copies of norms its rel-err sums are spread over (>= 1)
};

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

// ---------------------------------------------------------------------------------------
// The fused tile: load -> Y -> n_it TV iterations in registers -> store core.
// ---------------------------------------------------------------------------------------
struct TvShared {
    float ylds[TV_ROWS][TV_COLS];     // Y of the tile (prox anchor; tau*Y enters every iteration)
    float4 zrow[TV_NW][WAVE];         // first-row z of each wave (read by the wave above)
    float4 urow[TV_NW][WAVE];         // last-row u2[...,0] of each wave (read by the wave below)
    float red[MAXIT][TV_NW][2];       // per-wave rel_err partial sums
};

template <bool EXACT, int FRONT, bool ALPHA1>
__device__ __forceinline__ void tv_tile(const TvArgs& a, int plane, int tile, int n_it, bool track,
                                        long long step, bool fresh, TvShared& sh) {
    float4 (*zrow)[WAVE] = sh.zrow;
    float4 (*urow)[WAVE] = sh.urow;
    float (*red)[TV_NW][2] = sh.red;
    constexpr int R = TV_R;
    const int lane = threadIdx.x & (WAVE - 1);
    const int w = threadIdx.x >> 6;
    const int H = a.H, W = a.W, C = a.C;
    const int b = plane / C, c = plane - b * C;
    const int band = tile / a.nsegs, seg = tile - band * a.nsegs;
    const int r0 = band * a.band_h, r1 = min(H, r0 + a.band_h);
    const int e0 = max(0, r0 - a.halo), e1 = min(H, r1 + a.halo);
    const int cc0 = seg * a.seg_w, cc1 = min(W, cc0 + a.seg_w);
    const int f0 = max(0, cc0 - a.halo) & ~3;
    const int gj0 = f0 + CPL * lane;
    const size_t HW = (size_t)H * W;
    const size_t E = (size_t)C * HW;
    const size_t BE = (size_t)a.B * E;
    const size_t chain_off = (size_t)b * E;
    const size_t plane_off = chain_off + (size_t)c * HW;
    const bool vec = (W & 3) == 0;

    const int par_in = a.pingpong ? (int)(step & 1) : 0;
    const int par_out = a.pingpong ? (int)((step + 1) & 1) : 1;

    float x2[R][CPL], u0[R][CPL], u1[R][CPL], z[R][CPL];
    int gi[R];
    bool hasUp[R], hasDown[R];
    bool hasLeft[CPL], hasRight[CPL], colok[CPL], colcore[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int gj = gj0 + k;
        colok[k] = gj < W;
        hasLeft[k] = gj > 0;
        hasRight[k] = gj < W - 1;
        colcore[k] = gj >= cc0 && gj < cc1;
    }

    // ------------------------------ load + data term + noise ------------------------------
#pragma unroll
    for (int r = 0; r < R; ++r) {
        gi[r] = e0 + w * R + r;
        const bool rv = gi[r] < e1;
        hasUp[r] = gi[r] > 0;
        hasDown[r] = gi[r] < H - 1;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            x2[r][k] = 0.f; u0[r][k] = 0.f; u1[r][k] = 0.f; z[r][k] = 0.f;
        }
        float4 yst = make_float4(0.f, 0.f, 0.f, 0.f);
        if (rv && gj0 < W) {
            const size_t base = plane_off + (size_t)gi[r] * W + gj0;
            float Yv[CPL], xs[CPL], us0[CPL], us1[CPL];
            if (FRONT == FRONT_INPAINT) {
                float X[CPL], yo[CPL], mk[CPL], Z[CPL];
                const float* xin = a.x[par_in];
                const float* yb = a.yobs + (size_t)b * a.y_cs + (size_t)c * HW + (size_t)gi[r] * W + gj0;
                const uint8_t* mb = a.mask + (size_t)b * a.m_cs + (size_t)gi[r] * W + gj0;
                if (vec) {
                    const float4 xv = ld4(xin + base);
                    const float4 yy = ld4(yb);
                    const uchar4 mm = *reinterpret_cast<const uchar4*>(mb);
                    X[0] = xv.x; X[1] = xv.y; X[2] = xv.z; X[3] = xv.w;
                    yo[0] = yy.x; yo[1] = yy.y; yo[2] = yy.z; yo[3] = yy.w;
                    mk[0] = (float)mm.x; mk[1] = (float)mm.y; mk[2] = (float)mm.z; mk[3] = (float)mm.w;
                    const size_t e = ((size_t)c * H + gi[r]) * W + gj0;
                    normal_quad(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step, TAG_LANGEVIN,
                                (uint32_t)(e >> 2), Z);
                } else {
#pragma unroll
                    for (int k = 0; k < CPL; ++k) {
                        const bool ok = colok[k];
                        X[k] = ok ? xin[base + k] : 0.f;
                        yo[k] = ok ? yb[k] : 0.f;
                        mk[k] = ok ? (float)mb[k] : 0.f;
                        const size_t e = ((size_t)c * H + gi[r]) * W + gj0 + k;
                        Z[k] = ok ? normal_elem(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step,
                                                TAG_LANGEVIN, e)
                                  : 0.f;
                    }
                }
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    // g = ((-m) * (x - y)) / sigma2 ; Y = (X + c1 g) + c2 Z
                    const float g = (-mk[k] * (X[k] - yo[k])) / a.sigma2;
                    Yv[k] = (X[k] + a.c1 * g) + a.c2 * Z[k];
                    xs[k] = X[k];
                }
                if (!fresh && !ALPHA1) {
                    const float* x2in = a.x2[par_in];
                    if (vec) {
                        const float4 v = ld4(x2in + base);
                        xs[0] = v.x; xs[1] = v.y; xs[2] = v.z; xs[3] = v.w;
                    } else {
#pragma unroll
                        for (int k = 0; k < CPL; ++k) xs[k] = colok[k] ? x2in[base + k] : 0.f;
                    }
                }
            } else {  // FRONT_GIVEN: standalone prox of a given tensor
                const float* yin = a.yin;
                const float* x2in = a.x2[0];
                if (vec) {
                    const float4 v = ld4(yin + base);
                    Yv[0] = v.x; Yv[1] = v.y; Yv[2] = v.z; Yv[3] = v.w;
                    if (!fresh) {
                        const float4 q = ld4(x2in + base);
                        xs[0] = q.x; xs[1] = q.y; xs[2] = q.z; xs[3] = q.w;
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < CPL; ++k) {
                        Yv[k] = colok[k] ? yin[base + k] : 0.f;
                        if (!fresh) xs[k] = colok[k] ? x2in[base + k] : 0.f;
                    }
                }
            }
            if (!fresh) {
                const float* u2in = a.u2[par_in];
                if (vec) {
                    const float4 p = ld4(u2in + 2 * base);
                    const float4 q = ld4(u2in + 2 * base + 4);
                    us0[0] = p.x; us1[0] = p.y; us0[1] = p.z; us1[1] = p.w;
                    us0[2] = q.x; us1[2] = q.y; us0[3] = q.z; us1[3] = q.w;
                } else {
#pragma unroll
                    for (int k = 0; k < CPL; ++k) {
                        us0[k] = colok[k] ? u2in[2 * (base + k)] : 0.f;
                        us1[k] = colok[k] ? u2in[2 * (base + k) + 1] : 0.f;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                if (!colok[k]) continue;
                x2[r][k] = fresh ? Yv[k] : xs[k];
                u0[r][k] = fresh ? 0.f : us0[k];
                u1[r][k] = fresh ? 0.f : us1[k];
            }
            yst = make_float4(colok[0] ? Yv[0] : 0.f, colok[1] ? Yv[1] : 0.f, colok[2] ? Yv[2] : 0.f,
                              colok[3] ? Yv[3] : 0.f);
        }
        *reinterpret_cast<float4*>(&sh.ylds[w * R + r][CPL * lane]) = yst;
    }

    urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
    __syncthreads();

    // ------------------------------ inner TV iterations ------------------------------
    for (int it = 0; it < n_it; ++it) {
        const bool trk = track && it >= trk_lo(a) && it <= trk_hi(a);
        float sd = 0.f, sn = 0.f;
        // Phase A: x = prox_tau_fx(x2 - tau nabla^T u2, y); z = 2x - x2; x2 += rho (x - x2)
        const float4 up = (w > 0) ? urow[w - 1][lane] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float u1l = __shfl_up(u1[r][CPL - 1], 1);
            const float4 yrow = *reinterpret_cast<const float4*>(&sh.ylds[w * R + r][CPL * lane]);
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const float u0up = (r > 0) ? u0[r - 1][k] : f4get(up, k);
                const float u1left = (k > 0) ? u1[r][k - 1] : u1l;
                // nabla_adjoint in deepinv's order: ((0 - u0) + u0[i-1]) - u1) + u1[j-1]
                float t = hasDown[r] ? (0.0f - u0[r][k]) : 0.0f;
                t = hasUp[r] ? t + u0up : t;
                t = hasRight[k] ? t - u1[r][k] : t;
                t = hasLeft[k] ? t + u1left : t;
                const float xo = x2[r][k];
                float xv, zv, xn;
                if (EXACT) {
                    xv = ((xo - a.tau * t) + a.tau * f4get(yrow, k)) / a.opt;
                    zv = 2.0f * xv - xo;
                    xn = xo + a.rho * (xv - xo);
                } else {
                    xv = __builtin_fmaf(a.tau, f4get(yrow, k) - t, xo) * a.inv_opt;
                    zv = __builtin_fmaf(2.0f, xv, -xo);
                    xn = __builtin_fmaf(a.rho, xv - xo, xo);
                }
                if (trk) {
                    const bool core = colcore[k] && gi[r] >= r0 && gi[r] < r1;
                    const float d = xo - xn;
                    const float q = xn + 1e-12f;
                    sd += core ? d * d : 0.f;
                    sn += core ? q * q : 0.f;
                }
                z[r][k] = zv;
                x2[r][k] = xn;
            }
        }
        zrow[w][lane] = make_float4(z[0][0], z[0][1], z[0][2], z[0][3]);
        if (trk) {
            sd = wave_sum(sd);
            sn = wave_sum(sn);
            if (lane == 0) { red[it][w][0] = sd; red[it][w][1] = sn; }
        }
        __syncthreads();
        // Phase B: u = prox_sigma_g_conj(u2 + sigma nabla z, ths); u2 += rho (u - u2)
        const float4 dn = (w < TV_NW - 1) ? zrow[w + 1][lane] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float zr3 = __shfl_down(z[r][0], 1);
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const float zc = z[r][k];
                const float zd = (r < R - 1) ? z[r + 1][k] : f4get(dn, k);
                const float zr = (k < CPL - 1) ? z[r][k + 1] : zr3;
                const float g0 = hasDown[r] ? ((0.0f - zc) + zd) : 0.0f;
                const float g1 = hasRight[k] ? ((0.0f - zc) + zr) : 0.0f;
                const float uo0 = u0[r][k], uo1 = u1[r][k];
                if (EXACT) {
                    const float v0 = uo0 + a.sig_tv * g0;
                    const float v1 = uo1 + a.sig_tv * g1;
                    const float nrm = sqrtf(v0 * v0 + v1 * v1) / a.ths;
                    const float dd = fmaxf(nrm, 1.0f);
                    const float n0 = v0 / dd, n1 = v1 / dd;
                    u0[r][k] = uo0 + a.rho * (n0 - uo0);
                    u1[r][k] = uo1 + a.rho * (n1 - uo1);
                } else {
                    const float v0 = __builtin_fmaf(a.sig_tv, g0, uo0);
                    const float v1 = __builtin_fmaf(a.sig_tv, g1, uo1);
                    const float s2 = __builtin_fmaf(v0, v0, v1 * v1);
                    const float f = fminf(1.0f, a.ths * __builtin_amdgcn_rsqf(s2));
                    u0[r][k] = __builtin_fmaf(a.rho, __builtin_fmaf(v0, f, -uo0), uo0);
                    u1[r][k] = __builtin_fmaf(a.rho, __builtin_fmaf(v1, f, -uo1), uo1);
                }
            }
        }
        urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
        __syncthreads();
    }

    // rel_err partial sums -> global (one fp64 atomic per iteration and workgroup)
    if (track) {
        const int t = threadIdx.x;
        if (t >= trk_lo(a) && t <= trk_hi(a) && t < n_it) {
            double sd = 0.0, sn = 0.0;
            for (int ww = 0; ww < TV_NW; ++ww) { sd += red[t][ww][0]; sn += red[t][ww][1]; }
            const int g = a.per_chain_norm ? b : 0;
            atomicAdd(&a.norms[((size_t)g * a.n_tv + t) * 2], sd);
            atomicAdd(&a.norms[((size_t)g * a.n_tv + t) * 2 + 1], sn);
        }
    }

    // ------------------------------ store the core ------------------------------
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (gi[r] < r0 || gi[r] >= r1) continue;
        const size_t base = plane_off + (size_t)gi[r] * W + gj0;
        float Xo[CPL];
        const float4 yrow = *reinterpret_cast<const float4*>(&sh.ylds[w * R + r][CPL * lane]);
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            // X = (1 - alpha) Y + alpha D(Y)  (restoration_algorithms.py:238); alpha == 1 gives D(Y) exactly
            if (FRONT == FRONT_INPAINT && !ALPHA1)
                Xo[k] = (1.0f - a.alpha) * f4get(yrow, k) + a.alpha * x2[r][k];
            else
                Xo[k] = x2[r][k];
        }
        float* xout = (FRONT == FRONT_INPAINT) ? a.x[par_out] : a.x2[1];
        float* u2out = a.u2[par_out];
        if (vec && colcore[0]) {
            st4(xout + base, Xo[0], Xo[1], Xo[2], Xo[3]);
            st4(u2out + 2 * base, u0[r][0], u1[r][0], u0[r][1], u1[r][1]);
            st4(u2out + 2 * base + 4, u0[r][2], u1[r][2], u0[r][3], u1[r][3]);
            if (FRONT == FRONT_INPAINT && !ALPHA1)
                st4(a.x2[par_out] + base, x2[r][0], x2[r][1], x2[r][2], x2[r][3]);
        } else if (!vec) {
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                if (!colcore[k]) continue;
                xout[base + k] = Xo[k];
                u2out[2 * (base + k)] = u0[r][k];
                u2out[2 * (base + k) + 1] = u1[r][k];
                if (FRONT == FRONT_INPAINT && !ALPHA1) a.x2[par_out][base + k] = x2[r][k];
            }
        }
        if (FRONT == FRONT_INPAINT) {
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                if (!colcore[k]) continue;
                const size_t idx = base + k;   // == chain*E + e
                accumulate_elem(a, step, idx, BE, Xo[k], a.mean[par_in], a.sq[par_in], a.mean[par_out],
                                a.sq[par_out]);
            }
        }
    }
    (void)chain_off;
}

template <bool EXACT, int FRONT, bool ALPHA1>
__global__ void __launch_bounds__(TV_THREADS) tv_main_kernel(const TvArgs a) {
    __shared__ TvShared sh;
    const long long step = (a.d_step ? *a.d_step : 0LL) + a.step_offset;
    const bool fresh = a.fresh_dev ? (*a.fresh_dev != 0) : (a.fresh_host != 0);
    const int P = a.B * a.C;
    const int T = a.tiles;
    // XCD-aware order: blocks x and x+8 share an XCD (round-robin dispatch), so all
    // tiles of one plane land on one XCD and their halo rows hit that XCD's L2.
    const int x = blockIdx.x;
    const int xcd = x & 7;
    const int k = x >> 3;
    const int plane = (k / T) * 8 + xcd;
    const int tile = k - (k / T) * T;
    if (plane >= P) return;
    tv_tile<EXACT, FRONT, ALPHA1>(a, plane, tile, a.n_tv, true, step, fresh, sh);
}

// Early-stop finaliser (deepinv: break when rel_err < tol at inner iteration >= 2): recompute
// the tiles of the affected chains with the right number of inner iterations, then reset the
// workspace, clear the restart flag and advance the step counter (last block to arrive).
template <bool EXACT, int FRONT, bool ALPHA1>
__global__ void __launch_bounds__(TV_THREADS) tv_finalise_kernel(const TvArgs a) {
    __shared__ TvShared sh;
    __shared__ int s_stop[MAXG];
    __shared__ int s_flag;
    const long long step = (a.d_step ? *a.d_step : 0LL) + a.step_offset;
    const bool fresh = a.fresh_dev ? (*a.fresh_dev != 0) : (a.fresh_host != 0);
    const int P = a.B * a.C;
    const int T = a.tiles;
    const int G = a.per_chain_norm ? a.B : 1;
    if (threadIdx.x == 0) s_flag = 0;
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
        // all partial norms of the chain in flight at once (one memory latency, not n_tv)
        double nd[MAXIT], nn[MAXIT];
        const int tlo = trk_lo(a), thi = trk_hi(a);
#pragma unroll
        for (int t = 0; t < MAXIT; ++t) {
            if (t >= tlo && t <= thi) {
                nd[t] = a.norms[((size_t)g * a.n_tv + t) * 2];
                nn[t] = a.norms[((size_t)g * a.n_tv + t) * 2 + 1];
            }
        }
        int stop = a.n_tv;
        bool found = false;
#pragma unroll
        for (int t = 0; t < MAXIT; ++t) {
            if (t >= tlo && t <= thi && !found) {
                const float rel = (float)sqrt(nd[t]) / (float)sqrt(nn[t]);
                if (rel < a.tol) { stop = t + 1; found = true; }
            }
        }
        if (a.stopped && blockIdx.x == 0) a.stopped[g] = found ? stop : 0;
        s_stop[g] = stop;
        if (stop < a.n_tv) atomicOr(&s_flag, 1);
    }
    __syncthreads();
    if (s_flag) {
        for (int item = blockIdx.x; item < P * T; item += gridDim.x) {
            const int plane = item / T, tile = item - (item / T) * T;
            const int g = a.per_chain_norm ? plane / a.C : 0;
            if (s_stop[g] < a.n_tv) tv_tile<EXACT, FRONT, ALPHA1>(a, plane, tile, s_stop[g], false, step, fresh, sh);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const int old = atomicAdd(a.arrive, 1);
        s_flag = (old == (int)gridDim.x - 1) ? 2 : 0;
    }
    __syncthreads();
    if (s_flag == 2) {
        __threadfence();
        const int n = G * a.n_tv * 2;
        for (int i = threadIdx.x; i < n; i += blockDim.x) a.norms[i] = 0.0;
        if (threadIdx.x == 0) {
            *a.arrive = 0;
            if (a.fresh_dev) *a.fresh_dev = 0;
            if (a.advance_step && a.d_step) *a.d_step = step - a.step_offset + 1;   // the value read at the start: no dependent load
        }
    }
}

// ---------------------------------------------------------------------------------------
// Row-streaming pipeline: the production PSGLA+TV step for W % 4 == 0 and n_tv <= 10.
//
// One workgroup streams one (chain, channel) plane -- or a <=256-column segment of it, with
// a horizontal halo of n_tv columns -- from top to bottom, one row per pipeline step:
//   waves 0-3   FRONT: row r is owned by wave r % 4 and processed over 4 steps (software
//               pipelined): Philox, Box-Muller pair 1, pair 2, then the data term
//               Y = (X + c1 g) + c2 Z and the TV state (x2, u2) are written to LDS ring 0;
//               the global loads of the wave's next row are issued 4 steps ahead.
//   waves 4..   STAGE k = 1..n_tv (one wave per inner TV iteration): at step t it computes
//               the primal update of row j = t-2-2k and the dual update of row i = j-1 from
//               ring k-1 (written one step earlier) and writes (x2, u2) of row i to ring k.
//               Row i's dual update needs z of rows i and i+1, hence the lag of 2 per stage.
//   last 2      BACK: X = x2 (or the alpha relaxation), block accumulators, sample / block
//               slots, chain state out; mean/sq loads prefetched 2 rows ahead.
// All waves meet at one barrier per step.  Compared with the band kernel there is no
// vertical halo recompute, and the HBM loads / stores of every row overlap the TV
// iterations of the rows in flight (the band kernel runs load -> compute -> store in
// lockstep on every CU).
// ---------------------------------------------------------------------------------------
constexpr int SP_FRONT = 4;
constexpr int SP_BACK = 2;
constexpr int SP_MAXST = 10;
constexpr int SP_YRING = 32;
constexpr int SP_MAXSEG = 4;      // planes touched by one workgroup's row stream (split mode)
constexpr int SP_NOSEG = 1 << 30; // "no further segment start"

struct StreamShared {
    float4 x2[SP_MAXST + 1][2][WAVE];     // ring k = output of stage k (k = 0: front), 2 row slots
    float4 u0[SP_MAXST + 1][2][WAVE];
    float4 u1[SP_MAXST + 1][2][WAVE];
    float4 y[SP_YRING][WAVE];             // Y rows (prox anchor), alive from the front to the back
    // LDS-DMA staging (global_load_lds_dwordx4): a front wave's next row (X, y, u2 lo/hi, x2)
    // and a back wave's next mean/sq rows land here without occupying VGPRs.
    float4 fst[SP_FRONT][2][5][WAVE];
    uint32_t fmk[SP_FRONT][2][WAVE];
    float4 bst[SP_BACK][2][2][WAVE];
    float red[SP_MAXSEG][SP_MAXST][2];
};

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

// Row stream of a workgroup.  Per-plane mode: one segment = rows 0..H-1 of one plane.
// Split mode (row_split > 0): the P*H rows of all planes, concatenated, are cut into equal
// contiguous ranges of CORE rows, one per workgroup, so that every CU gets work even when
// P < #CUs.  A range may span several planes (segments, at most SP_MAXSEG); where it starts or
// ends inside a plane it is extended by n_tv halo rows, which are computed (with the plane
// edge treated as a boundary) but neither stored nor counted: the TV dependency cone grows by
// one row per inner iteration, so after n_tv iterations the core rows are exact.  Interior
// segment boundaries are true plane edges.  All fields are workgroup-uniform (SGPRs).
struct RowMap {
    int ns;                      // segments (1 .. SP_MAXSEG)
    int Q;                       // stream rows (halo included)
    int htop, hbot;              // halo rows at the start / end of the stream
    int q1, q2, q3;              // stream index of segments 1..3 (Q when absent); segment 0 starts at 0
    int pl0, pl1, pl2, pl3;      // plane of each segment
    int lo0, lo1, lo2, lo3;      // plane row of each segment's first stream row
    // (scalar members, not arrays: the struct must stay in SGPRs)
    __device__ __forceinline__ int qs(int s) const { return s <= 0 ? 0 : (s == 1 ? q1 : (s == 2 ? q2 : (s == 3 ? q3 : Q))); }
    __device__ __forceinline__ int pl(int s) const { return s == 0 ? pl0 : (s == 1 ? pl1 : (s == 2 ? pl2 : pl3)); }
    __device__ __forceinline__ int lo(int s) const { return s == 0 ? lo0 : (s == 1 ? lo1 : (s == 2 ? lo2 : lo3)); }
};

__device__ __forceinline__ void build_rowmap(const TvArgs& a, int wg, RowMap& m) {
    const int H = a.H;
    m.pl0 = m.pl1 = m.pl2 = m.pl3 = 0;
    m.lo0 = m.lo1 = m.lo2 = m.lo3 = 0;
    if (a.split_wgs <= 0) {
        m.ns = 1; m.Q = H; m.htop = 0; m.hbot = 0;
        m.q1 = m.q2 = m.q3 = H;
        m.pl0 = wg;                   // virtual plane (plane * st_nsegs + column segment)
        return;
    }
    const long long T = (long long)a.B * a.C * a.st_nsegs * H;
    const long long g0 = T * wg / a.split_wgs, g1 = T * (wg + 1) / a.split_wgs;
    const int p0 = (int)(g0 / H), p1 = (int)((g1 - 1) / H);
    const int h = a.n_tv;
    m.ns = p1 - p0 + 1;
    // segment s covers plane p0 + s; only the first can start and the last can end inside it
    auto seg = [&](int s, int& lo, int& len, int& ht, int& hb) {
        const int p = p0 + s;
        const int clo = (s == 0) ? (int)(g0 - (long long)p * H) : 0;
        const int chi = (p == p1) ? (int)(g1 - (long long)p * H) : H;
        lo = clo > 0 ? max(0, clo - h) : 0;
        const int hi = chi < H ? min(H, chi + h) : H;
        len = hi - lo;
        ht = clo - lo;
        hb = hi - chi;
    };
    int lo, len, ht, hb;
    seg(0, lo, len, ht, hb);
    m.pl0 = p0; m.lo0 = lo; m.htop = ht; m.hbot = hb;
    int q = len;
    m.q1 = m.q2 = m.q3 = 0;
    if (m.ns > 1) { seg(1, lo, len, ht, hb); m.q1 = q; m.pl1 = p0 + 1; m.lo1 = lo; m.hbot = hb; q += len; }
    if (m.ns > 2) { seg(2, lo, len, ht, hb); m.q2 = q; m.pl2 = p0 + 2; m.lo2 = lo; m.hbot = hb; q += len; }
    if (m.ns > 3) { seg(3, lo, len, ht, hb); m.q3 = q; m.pl3 = p0 + 3; m.lo3 = lo; m.hbot = hb; q += len; }
    m.Q = q;
    if (m.ns <= 1) m.q1 = q;
    if (m.ns <= 2) m.q2 = q;
    if (m.ns <= 3) m.q3 = q;
}

// One whole plane (the early-stop recompute pass).
__device__ __forceinline__ void plane_rowmap(int H, int plane, RowMap& m) {
    m.ns = 1; m.Q = H; m.htop = 0; m.hbot = 0;
    m.q1 = m.q2 = m.q3 = H;
    m.pl0 = plane; m.pl1 = m.pl2 = m.pl3 = 0;
    m.lo0 = m.lo1 = m.lo2 = m.lo3 = 0;
}

// Column geometry of a virtual plane vp = plane * st_nsegs + segment: the real plane, the start of the
// segment's 256-column wave window (f0) and its core columns [cc0, cc1).  Without GEN there is one
// segment (vp = plane, the whole row).
struct SegGeo {
    int rp, f0, cc0, cc1;
};
template <bool GEN>
__device__ __forceinline__ SegGeo seg_geo(const TvArgs& a, int vp) {
    SegGeo g;
    if (!GEN) {
        g.rp = vp; g.f0 = 0; g.cc0 = 0; g.cc1 = a.W;
        return g;
    }
    const int ns = a.st_nsegs;
    g.rp = vp / ns;
    const int sgi = vp - g.rp * ns;
    g.cc0 = sgi * a.st_seg_w;
    g.cc1 = min(a.W, g.cc0 + a.st_seg_w);
    g.f0 = max(0, g.cc0 - a.st_halo) & ~3;
    return g;
}

// Position of a role's current row in the stream; advanced monotonically (the segment walk
// runs only when a plane boundary is crossed).
struct RowCursor {
    int q, s, p, r, qend;
};
__device__ __forceinline__ void cursor_seek(const RowMap& m, RowCursor& c) {
    while (c.s + 1 < m.ns && c.q >= m.qs(c.s + 1)) ++c.s;
    c.qend = m.qs(c.s + 1);
    c.p = m.pl(c.s);
    c.r = m.lo(c.s) + (c.q - m.qs(c.s));
}
__device__ __forceinline__ void cursor_init(const RowMap& m, RowCursor& c, int q) {
    c.q = q; c.s = 0;
    cursor_seek(m, c);
}
__device__ __forceinline__ void cursor_advance(const RowMap& m, RowCursor& c, int d) {
    c.q += d; c.r += d;
    if (c.q >= c.qend && c.s + 1 < m.ns) cursor_seek(m, c);
}
// stream index of the first segment start after stream row q (SP_NOSEG if none)
__device__ __forceinline__ int next_seg_start(const RowMap& m, int q) {
    if (m.ns > 1 && m.q1 > q) return m.q1;
    if (m.ns > 2 && m.q2 > q) return m.q2;
    if (m.ns > 3 && m.q3 > q) return m.q3;
    return SP_NOSEG;
}

// One pipeline stage = one inner TV iteration on one row pair.  Phase A (primal) on the
// lookahead row j from ring k-1; phase B (dual) on the output row i = j-1, which needs z of
// rows i (held from the previous step) and j.
struct StageRow {
    float u0[CPL], u1[CPL];   // u2^{k-1} of the row
    float z[CPL];             // z^k of the row
    float x2n[CPL];           // x2^k of the row
    int lk;                   // GEN: the row's lastk (its column segment's), set by the primal
};

template <bool EXACT, bool TRK, bool GEN = false>
__device__ __forceinline__ void stage_phase_a(const TvArgs& a, const float4& X2, const float4& U0,
                                              const float4& U1, const float4& YY, const float (&pu0)[CPL],
                                              StageRow& o, float& sd, float& sn, int nreal = CPL) {
    const float x2o[CPL] = {X2.x, X2.y, X2.z, X2.w};
    const float yy[CPL] = {YY.x, YY.y, YY.z, YY.w};
    o.u0[0] = U0.x; o.u0[1] = U0.y; o.u0[2] = U0.z; o.u0[3] = U0.w;
    o.u1[0] = U1.x; o.u1[1] = U1.y; o.u1[2] = U1.z; o.u1[3] = U1.w;
    // u1 of the column left of this lane's first column (lane-1's last); 0 at lane 0
    const float u1l = __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(o.u1[CPL - 1]), 0x138 /* wave_shr:1 */, 0xF, 0xF, true));
#pragma unroll
    for (int kk = 0; kk < CPL; ++kk) {
        const float u1left = kk > 0 ? o.u1[kk - 1] : u1l;
        // nabla^T u2 in deepinv's order: (((0 - u0) + u0[i-1]) - u1) + u1[j-1]; 0 - u0 + p == p - u0
        // exactly (up to the sign of a zero, which no later operation can observe)
        const float tt = ((pu0[kk] - o.u0[kk]) - o.u1[kk]) + u1left;
        const float xo = x2o[kk];
        float xv, zv, xn;
        if (EXACT) {
            xv = ((xo - a.tau * tt) + a.tau * yy[kk]) / a.opt;
            zv = 2.0f * xv - xo;
            xn = xo + a.rho * (xv - xo);
        } else {
            xv = __builtin_fmaf(a.tau, yy[kk] - tt, xo) * a.inv_opt;
            zv = __builtin_fmaf(2.0f, xv, -xo);
            xn = __builtin_fmaf(a.rho, xv - xo, xo);
        }
        if (TRK) {
            // padded rows (GEN): the lane's columns >= W are not part of the image's norms
            const bool real = !GEN || kk < nreal;
            if (EXACT) {
                const float d = real ? xo - xn : 0.f;
                const float q = real ? xn + 1e-12f : 0.f;
                sd = __builtin_fmaf(d, d, sd);
                sn = __builtin_fmaf(q, q, sn);
            } else {
                // ||x2_prev - x2|| = rho ||x - x2_prev||: accumulate (x - x2_prev)^2, scaled by rho^2
                // when the sums are published; the +1e-12 of ||x2 + 1e-12|| is below fp32 resolution
                // of any pixel value that contributes
                const float d = real ? xv - xo : 0.f;
                const float q = real ? xn : 0.f;
                sd = __builtin_fmaf(d, d, sd);
                sn = __builtin_fmaf(q, q, sn);
            }
        }
        o.z[kk] = zv;
        o.x2n[kk] = xn;
    }
}

// lastk: index (0..3) of the image's last column among this lane's columns, else outside 0..3
// (GEN = false: the image's last column is always the last one of a lane)
template <bool EXACT, bool DN, bool GEN = false>
__device__ __forceinline__ void stage_phase_b(const TvArgs& a, const StageRow& ri, const float (&zj)[CPL],
                                              int lastk, float (&un0)[CPL], float (&un1)[CPL]) {
    // z of the column right of this lane's last column (lane+1's first)
    const float zr3 = __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(ri.z[0]), 0x130 /* wave_shl:1 */, 0xF, 0xF, true));
#pragma unroll
    for (int kk = 0; kk < CPL; ++kk) {
        const float zc = ri.z[kk];
        const float zr = kk < CPL - 1 ? ri.z[kk + 1] : zr3;
        // deepinv: (0 - z) + z_next == z_next - z exactly (up to the sign of a zero)
        const float g0 = DN ? (zj[kk] - zc) : 0.0f;
        float g1 = zr - zc;
        if (GEN || kk == CPL - 1) g1 = (lastk == kk) ? 0.0f : g1;
        const float uo0 = ri.u0[kk], uo1 = ri.u1[kk];
        if (EXACT) {
            const float v0 = uo0 + a.sig_tv * g0;
            const float v1 = uo1 + a.sig_tv * g1;
            const float nrm = sqrtf(v0 * v0 + v1 * v1) / a.ths;
            const float dd = fmaxf(nrm, 1.0f);
            un0[kk] = uo0 + a.rho * (v0 / dd - uo0);
            un1[kk] = uo1 + a.rho * (v1 / dd - uo1);
        } else {
            const float v0 = __builtin_fmaf(a.sig_tv, g0, uo0);
            const float v1 = __builtin_fmaf(a.sig_tv, g1, uo1);
            const float s2 = __builtin_fmaf(v0, v0, v1 * v1);
            const float f = fminf(1.0f, a.ths * __builtin_amdgcn_rsqf(s2));
            un0[kk] = __builtin_fmaf(a.rho, __builtin_fmaf(v0, f, -uo0), uo0);
            un1[kk] = __builtin_fmaf(a.rho, __builtin_fmaf(v1, f, -uo1), uo1);
        }
    }
}

// Stage k's whole life over the row stream.  At step t the stage (lookahead row j = t - 3k - 1)
//   1. issues the LDS reads of ring k-1 row j,
//   2. runs the dual update of row i = j - 2 -- every input is already in registers (z of
//      rows i and i+1 from the two previous steps) -- and writes row i to ring k,
//   3. runs the primal update of row j once the reads have landed.
// The ring reads' latency and the ring writes thus overlap computation instead of
// bracketing it.  Three row states rotate (RA -> RB -> RC) so nothing is copied.
// Segment edges (split mode): the first row of a segment has no row above (its primal
// uses u0 = 0 above) and the last has no row below (its dual has no vertical difference);
// the rel-err partial sums are flushed per segment (different segments may be different chains).
template <bool EXACT, bool TRK, bool GEN>
__device__ __forceinline__ void stage_loop(const TvArgs& a, StreamShared& sh, const RowMap& rm, int k, int n,
                                           int nsteps, int Qk, int lane, int lastk, int nreal, bool core) {
    // GEN: the lane's columns change with the column segment of the row (row split over virtual
    // planes): lastk / nreal / core follow the primal row's segment; each row carries its lastk
    // to its dual (StageRow.lk)
    auto set_geo = [&](int sgi) {
        if (GEN) {
            const SegGeo g = seg_geo<GEN>(a, rm.pl(sgi));
            const int gj = g.f0 + CPL * lane;
            lastk = a.W - 1 - gj;
            nreal = min(CPL, max(0, a.W - gj));
            core = gj < a.W && gj >= g.cc0 && gj < g.cc1;
        }
    };
    const int Q = Qk;                    // rows this stage runs (the stream's, bottom-halo trimmed)
    const int tbeg = 1 + 3 * k;          // step of lookahead row 0
    StageRow RA, RB, RC;
    const float zero[CPL] = {0.f, 0.f, 0.f, 0.f};
    float lsd = 0.f, lsn = 0.f;          // rel-err partial sums of segment sacc (core rows)
    int sacc = 0;
    int nb = next_seg_start(rm, 0);      // next segment start after the current primal row
    bool fprev = false;                  // row j-1 started a segment
    const int qc0 = rm.htop, qc1 = Q - rm.hbot;   // core stream rows
    auto flush = [&]() {
        if (TRK) {
            float d = wave_sum(core ? lsd : 0.f);
            const float q = wave_sum(core ? lsn : 0.f);
            if (!EXACT) d *= a.rho * a.rho;          // fast sums hold (x - x2_prev)^2
            if (lane == 0) { sh.red[sacc][k - 1][0] = d; sh.red[sacc][k - 1][1] = q; }
            lsd = 0.f; lsn = 0.f;
        }
    };
    auto primal = [&](int j, const float4& X2, const float4& U0, const float4& U1, const float4& YY,
                      const float (&pu0)[CPL], StageRow& cur) {
        float rd = 0.f, rn = 0.f;
        stage_phase_a<EXACT, TRK, GEN>(a, X2, U0, U1, YY, pu0, cur, rd, rn, nreal);
        if (GEN) cur.lk = lastk;
        if (TRK && j >= qc0 && j < qc1) { lsd += rd; lsn += rn; }
    };
    int t = 0;
    for (; t < tbeg; ++t) step_barrier();
    auto load_row = [&](int j, float4& X2, float4& U0, float4& U1, float4& YY) {
        const int sl = j & 1;
        X2 = sh.x2[k - 1][sl][lane];
        U0 = sh.u0[k - 1][sl][lane];
        U1 = sh.u1[k - 1][sl][lane];
        YY = sh.y[j & (SP_YRING - 1)][lane];
    };
    auto store_row = [&](int i, const StageRow& r, const float (&un0)[CPL], const float (&un1)[CPL]) {
        const int so = i & 1;
        sh.x2[k][so][lane] = make_float4(r.x2n[0], r.x2n[1], r.x2n[2], r.x2n[3]);
        sh.u0[k][so][lane] = make_float4(un0[0], un0[1], un0[2], un0[3]);
        sh.u1[k][so][lane] = make_float4(un1[0], un1[1], un1[2], un1[3]);
    };
    // rows 0 and 1: primal update only (segments hold >= 2 rows: row 1 never starts one)
    {
        float4 X2, U0, U1, YY;
        load_row(0, X2, U0, U1, YY);
        primal(0, X2, U0, U1, YY, zero, RA);
        step_barrier();
        load_row(1, X2, U0, U1, YY);
        primal(1, X2, U0, U1, YY, RA.u0, RB);
        step_barrier();
        t += 2;
    }
    // middle rows j = 2..Q-1: dual update of row j-2 (p2) with z of row j-1 (p1), then primal of j
    auto middle = [&](int j, StageRow& p2, StageRow& p1, StageRow& cur) {
        float4 X2, U0, U1, YY;
        load_row(j, X2, U0, U1, YY);
        float un0[CPL], un1[CPL];
        if (!fprev) stage_phase_b<EXACT, true, GEN>(a, p2, p1.z, GEN ? p2.lk : lastk, un0, un1);
        else stage_phase_b<EXACT, false, GEN>(a, p2, zero, GEN ? p2.lk : lastk, un0, un1);   // row j-2 ends a segment
        store_row(j - 2, p2, un0, un1);
        const bool fj = j == nb;
        if (fj) {                       // row j starts a new segment (split mode only)
            flush();
            ++sacc;
            nb = next_seg_start(rm, j);
            set_geo(sacc);
            primal(j, X2, U0, U1, YY, zero, cur);
        } else {
            primal(j, X2, U0, U1, YY, p1.u0, cur);
        }
        fprev = fj;
        step_barrier();
    };
    int j = 2;
    for (; j + 2 < Q; j += 3) {
        middle(j, RA, RB, RC);
        middle(j + 1, RB, RC, RA);
        middle(j + 2, RC, RA, RB);
    }
    t += (j - 2);
    // j = Q: dual update of row Q-2 (z of row Q-1 known); j = Q+1: row Q-1 (no row below).
    // (static buffer roles per remainder: a runtime-indexed StageRow would go to scratch)
    auto finish = [&](StageRow& r2, StageRow& r1) {
        float un0[CPL], un1[CPL];
        stage_phase_b<EXACT, true, GEN>(a, r2, r1.z, GEN ? r2.lk : lastk, un0, un1);
        store_row(Q - 2, r2, un0, un1);
        step_barrier();
        stage_phase_b<EXACT, false, GEN>(a, r1, zero, GEN ? r1.lk : lastk, un0, un1);
        store_row(Q - 1, r1, un0, un1);
        step_barrier();
    };
    const int rem = Q - j;              // 0, 1 or 2 middle rows left
    if (rem == 0) {
        finish(RA, RB);
    } else if (rem == 1) {
        middle(j, RA, RB, RC);
        finish(RB, RC);
    } else {
        middle(j, RA, RB, RC);
        middle(j + 1, RB, RC, RA);
        finish(RC, RA);
    }
    t += rem + 2;
    for (; t < nsteps; ++t) step_barrier();
    flush();
}

// One pass of the row-streaming pipeline over the rows of `rm` with n inner TV iterations
// (front / stage / back roles, one barrier per step).  Inlined at two call sites: the main
// pass and the rare early-stop recompute, each with its own register allocation.
// GEN: the row pitch is not the image width (rows padded: W % 4 != 0) -- the last-column, norm
// and noise-window handling of such rows, compiled only into the kernels that need it
template <bool EXACT, bool ALPHA1, bool GEN>
__device__ __forceinline__ void stream_pass(const TvArgs& a, StreamShared& sh, const RowMap& rm, const int n,
                                            const bool track, const long long step, const bool fresh) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (scalar branches)
    const int H = a.H, W = a.W, C = a.C;
    const int L = a.ldw;                                   // row pitch (memory); W: the image's width
    const size_t HW = (size_t)H * L;                       // plane pitch
    const size_t E = (size_t)C * HW;
    const size_t BE = (size_t)a.B * E;
    const int par_in = (int)(step & 1), par_out = (int)((step + 1) & 1);
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
    auto plane_off = [&](int pl) -> size_t { return (size_t)pl * HW; };   // planes are (b, c) in NCHW order
    const int Q = rm.Q;
    const int qc0 = rm.htop, qc1 = Q - rm.hbot;          // core stream rows
    // column geometry of the first row's segment (the only one without GEN)
    const SegGeo g0 = seg_geo<GEN>(a, rm.pl0);
    const int cc0 = g0.cc0, cc1 = g0.cc1;
    const int gj0 = g0.f0 + CPL * lane;
    const bool lane_ok = gj0 < W;
    const bool core = lane_ok && gj0 >= cc0 && gj0 < cc1;   // a lane's 4 columns are all core or none
    // Bottom-halo trim (split mode): the stream's last row is an artificial edge, so stage k's
    // output is exact down to one row less than its input's; the core rows (< Qb) only need
    // stage k to run rows 0 .. Qb + n - k, and the back none of the halo rows.  The pipeline
    // drains hbot - 1 steps earlier (no change without a bottom halo).
    const int Qb = Q - rm.hbot;
    auto stage_rows = [&](int k) { return min(Q, Qb + n - k + 1); };
    int nsteps = max(Q + 4, Qb + 4 + 3 * n);
    for (int k = 1; k <= n; ++k) nsteps = max(nsteps, stage_rows(k) + 3 + 3 * k);
    // 16 waves always; waves beyond the pipeline (n < 10) only keep the barrier count
    const int role = (w < SP_FRONT) ? 0 : (w < SP_FRONT + n ? 1 : (w < SP_FRONT + n + SP_BACK ? 2 : 3));

    const int k_st = w - SP_FRONT + 1;                 // inner TV iteration (1-based)
    const bool trk = track && role == 1 && (k_st - 1) >= 2 && (k_st - 1) <= n - 2;
    // Each role runs its own loop (its state is live only there); every wave executes
    // exactly nsteps barriers, so the s_barrier instances pair up across roles.
    if (role == 0) {
        // ---------------- FRONT state ----------------
        const int fw = w;                                  // front wave id (stream rows q % 4 == fw)
        uint32_t ph0 = 0, ph1 = 0, ph2 = 0, ph3 = 0;
        float zn0 = 0.f, zn1 = 0.f, zn2 = 0.f, zn3 = 0.f;
        uint32_t pq0 = 0, pq1 = 0, pq2 = 0, pq3 = 0;          // second quad (W % 4 != 0 rows)
        float zq0 = 0.f, zq1 = 0.f, zq2 = 0.f, zq3 = 0.f;
        int esh = 0;
        int gjf = gj0;                                      // first column of the lane in row q (GEN:
        bool okf = lane_ok;                                 // per column segment)
        const float* xin = a.x[par_in];
        const float* u2in = a.u2[par_in];
        const float* x2in = ALPHA1 ? nullptr : a.x2[par_in];
        // The loads of a row are LDS-DMA'd 4 steps before the row is consumed (double-buffered
        // per front wave), row and column clamped into the plane so every lane loads.
        const int gjc = min(gj0, L - CPL);
        RowCursor rc_cur, rc_dma;
        cursor_init(rm, rc_cur, min(fw, Q - 1));
        cursor_init(rm, rc_dma, min(fw, Q - 1));
        // part `part` of the loads of stream row q: 0 = X, 1 = y, 2 = u2 (two halves), 3 = mask (+ x2)
        auto front_issue = [&](int part, int q, const RowCursor& rc) {
            const int rr = min(rc.r, H - 1);
            const int bi = (q >> 2) & 1;
            const SegGeo g = seg_geo<GEN>(a, rc.p);
            const int gjr = GEN ? min(g.f0 + CPL * lane, L - CPL) : gjc;
            const int bb = g.rp / C;
            // 64-bit per-lane addresses (the SGPR-base form measured +12 % in round 2:
            // this kernel's row cursor sits in VGPRs, so each DMA pays two readfirstlane + 5 wait states)
            const size_t base = plane_off(g.rp) + (size_t)rr * L + gjr;
            if (part == 0) {
                glds16(xin + base, &sh.fst[fw][bi][0][0]);
            } else if (part == 1) {
                glds16(a.yobs + (size_t)bb * a.y_cs + (size_t)(g.rp - bb * C) * HW + (size_t)rr * L + gjr,
                       &sh.fst[fw][bi][1][0]);
            } else if (part == 2) {
                glds16(u2in + 2 * base, &sh.fst[fw][bi][2][0]);
                glds16(u2in + 2 * base + 4, &sh.fst[fw][bi][3][0]);
            } else {
                if (!ALPHA1) glds16(x2in + base, &sh.fst[fw][bi][4][0]);
                glds4(a.mask + (size_t)bb * a.m_cs + (size_t)rr * L + gjr, &sh.fmk[fw][bi][0]);
            }
        };
        // row fw's loads up front; afterwards the loads of row q + 4 are issued one part per
        // phase of row q (into the buffer of row q - 4, consumed before phase 0 of row q), so
        // their issue cost is spread over four steps
        for (int part = 0; part < 4; ++part) front_issue(part, fw, rc_dma);
        cursor_advance(rm, rc_dma, min(4, max(0, Q - 1 - fw)));
        for (int t = 0; t < nsteps; ++t) {
                // ======================= FRONT =======================
                const int p = (t + 4 - fw) & 3;
                const int q = t - p;
                if (q >= 0 && q < Q) {
                    if (p < 3) front_issue(p, q + 4, rc_dma);
                    if (p == 0) {
                        const SegGeo g = seg_geo<GEN>(a, rc_cur.p);
                        const int bb = g.rp / C, cc = g.rp - bb * C;
                        if (GEN) {                                  // this row's segment's lanes
                            gjf = g.f0 + CPL * lane;
                            okf = gjf < W;
                        }
                        // element index in the chain's unpadded C*H*W image: the noise stream
                        // does not depend on the row pitch
                        const size_t e = ((size_t)cc * H + rc_cur.r) * W + gjf;
                        esh = (int)(e & 3);                         // the same for every lane of the row
                        uint32_t c0 = (uint32_t)(e >> 2), c1 = (uint32_t)step, c2 = TAG_LANGEVIN,
                                 c3 = (uint32_t)(a.seed >> 32);
                        philox4x32_10(c0, c1, c2, c3, (uint32_t)a.seed, (uint32_t)(a.chain0 + bb));
                        ph0 = c0; ph1 = c1; ph2 = c2; ph3 = c3;
                        if (GEN && esh != 0) {                     // the lane's 4 elements span two quads
                            uint32_t d0 = (uint32_t)(e >> 2) + 1u, d1 = (uint32_t)step, d2 = TAG_LANGEVIN,
                                     d3 = (uint32_t)(a.seed >> 32);
                            philox4x32_10(d0, d1, d2, d3, (uint32_t)a.seed, (uint32_t)(a.chain0 + bb));
                            pq0 = d0; pq1 = d1; pq2 = d2; pq3 = d3;
                        }
                    } else if (p == 1) {
                        box_muller(ph0, ph1, zn0, zn1);
                        if (GEN && esh != 0) box_muller(pq0, pq1, zq0, zq1);
                    } else if (p == 2) {
                        box_muller(ph2, ph3, zn2, zn3);
                        if (GEN && esh != 0) {
                            box_muller(pq2, pq3, zq2, zq3);
                            // element i of the lane = output (esh + i) of the two-quad window
                            const float w8[8] = {zn0, zn1, zn2, zn3, zq0, zq1, zq2, zq3};
                            float r4[CPL];
#pragma unroll
                            for (int i = 0; i < CPL; ++i)
                                r4[i] = esh == 1 ? w8[i + 1] : (esh == 2 ? w8[i + 2] : w8[i + 3]);
                            zn0 = r4[0]; zn1 = r4[1]; zn2 = r4[2]; zn3 = r4[3];
                        }
                    } else {
                        wait_vm<ALPHA1 ? 4 : 4>();   // row q's loads landed; parts 0-2 of row q + 4 may fly
                        const int bi = (q >> 2) & 1;
                        const float4 fX = sh.fst[fw][bi][0][lane];
                        const float4 fYo = sh.fst[fw][bi][1][lane];
                        const float4 fU0 = sh.fst[fw][bi][2][lane];
                        const float4 fU1 = sh.fst[fw][bi][3][lane];
                        const float4 fXS = ALPHA1 ? zero4 : sh.fst[fw][bi][4][lane];
                        const uint32_t fMw = sh.fmk[fw][bi][lane];
                        const float X[CPL] = {fX.x, fX.y, fX.z, fX.w};
                        const float yo[CPL] = {fYo.x, fYo.y, fYo.z, fYo.w};
                        const float mk[CPL] = {(float)(fMw & 0xFFu), (float)((fMw >> 8) & 0xFFu),
                                               (float)((fMw >> 16) & 0xFFu), (float)(fMw >> 24)};
                        const float Z[CPL] = {zn0, zn1, zn2, zn3};
                        float Yv[CPL];
#pragma unroll
                        for (int k = 0; k < CPL; ++k) {
                            if (EXACT) {
                                const float g = (-mk[k] * (X[k] - yo[k])) / a.sigma2;
                                Yv[k] = okf ? (X[k] + a.c1 * g) + a.c2 * Z[k] : 0.f;
                            } else {
                                const float g = (mk[k] * (yo[k] - X[k])) * a.inv_sigma2;
                                Yv[k] = okf ? __builtin_fmaf(a.c2, Z[k], __builtin_fmaf(a.c1, g, X[k])) : 0.f;
                            }
                        }
                        const float4 Y4 = make_float4(Yv[0], Yv[1], Yv[2], Yv[3]);
                        float4 x2s;
                        if (fresh) x2s = Y4;
                        else x2s = ALPHA1 ? fX : fXS;
                        if (!okf) x2s = zero4;
                        const int s0 = q & 1;
                        sh.x2[0][s0][lane] = x2s;
                        sh.u0[0][s0][lane] = fresh ? zero4 : make_float4(fU0.x, fU0.z, fU1.x, fU1.z);
                        sh.u1[0][s0][lane] = fresh ? zero4 : make_float4(fU0.y, fU0.w, fU1.y, fU1.w);
                        sh.y[q & (SP_YRING - 1)][lane] = Y4;
                            // the wave's next rows: noise row q + 4, DMA of row q + 8... issued as q + 4
                        front_issue(3, q + 4, rc_dma);
                        cursor_advance(rm, rc_cur, 4);
                        if (q + 8 < Q) cursor_advance(rm, rc_dma, 4);
                    }
                }
            step_barrier();
        }
    } else if (role == 1) {
        // ---------------- STAGE (one inner TV iteration per wave) ----------------
        // the only column whose forward difference is forced to 0 is the image's right edge;
        // the left edge, the last row of u2[...,0] and the last column of u2[...,1] need no
        // select: the DPP shift feeds 0 at lane 0 and TV keeps those dual components exactly 0.
        const int lastk = W - 1 - gj0;                    // in 0..3 on the lane holding column W-1
        const int nreal = min(CPL, max(0, W - gj0));      // real (non-pitch-padding) columns of the lane
        __builtin_amdgcn_s_setprio(1);
        const int qk = stage_rows(k_st);
        if (trk) stage_loop<EXACT, true, GEN>(a, sh, rm, k_st, n, nsteps, qk, lane, lastk, nreal, core);
        else stage_loop<EXACT, false, GEN>(a, sh, rm, k_st, n, nsteps, qk, lane, lastk, nreal, core);
    } else if (role == 3) {
        for (int t = 0; t < nsteps; ++t) step_barrier();
    } else {
        // ---------------- BACK state ----------------
        const int bw = w - SP_FRONT - n;                   // back wave id (stream rows q % 2 == bw)
        // issue priority: back > stages > front.  The back waves are the youngest of the
        // workgroup (lowest age priority) yet close every step (its last arrivals, measured);
        // raising them, then the stages, cut the step by 9 % (A/B).
        __builtin_amdgcn_s_setprio(3);
        const StepInfo si = step_info(a, step, a.mean[par_out]);
        const float* mean_in = a.mean[par_in];
        const float* sq_in = a.sq[par_in];
        const bool need_prev = si.acc && !si.first;
        const int gjc = min(gj0, L - CPL);
        RowCursor rc_cur, rc_dma;
        cursor_init(rm, rc_cur, min(bw, Q - 1));
        cursor_init(rm, rc_dma, min(bw, Q - 1));
        auto back_issue = [&](int q, const RowCursor& rc) {
            if (need_prev) {
                const int rr = min(rc.r, H - 1);
                const int bi = (q >> 1) & 1;
                const SegGeo g = seg_geo<GEN>(a, rc.p);
                const int gjr = GEN ? min(g.f0 + CPL * lane, L - CPL) : gjc;
                const size_t base = plane_off(g.rp) + (size_t)rr * L + gjr;
                glds16(mean_in + base, &sh.bst[bw][bi][0][0]);
                glds16(sq_in + base, &sh.bst[bw][bi][1][0]);
            }
        };
        // vector-memory stores per core row (all lanes of a wave store together; lane 0 is core)
        const int nst = 3 + (ALPHA1 ? 0 : 1) + ((si.acc && (si.blockend || si.liveout)) ? 2 : 0) + (si.sample ? 1 : 0);
        // a row's stores are spread over the wave's two steps: state + accumulators, then the rest
        bool hold = false, hcore = core;
        size_t h_base = 0;                  // per-lane element index
        uint32_t h_vo = 0;                  // the lane's column as a byte offset
        float4 hM = zero4, hQ = zero4, hX = zero4;
        auto flush_held = [&]() {
            if (!(GEN ? hcore : core)) return;
            if (si.acc) {
                if (si.blockend) {
                    st_nt(a.blocks + (size_t)si.blk * BE + h_base, hM);
                    st_nt(a.blocks2 + (size_t)si.blk * BE + h_base, hQ);
                } else if (si.liveout) {
                    st_nt(a.mean[par_out] + h_base, hM);
                    st_nt(a.sq[par_out] + h_base, hQ);
                }
            }
            if (si.sample) st_nt(a.samples + (size_t)si.sidx * BE + h_base, hX);
        };
        // mean / sq rows are LDS-DMA'd two of the wave's rows ahead (4 stream rows); c1 / c2 =
        // vector-memory ops issued after the DMA of the wave's next / next-but-one row
        back_issue(bw, rc_dma);
        if (bw + 2 < Q) cursor_advance(rm, rc_dma, 2);
        back_issue(bw + 2, rc_dma);
        int c1 = 2, c2 = 0;
        for (int t = 0; t < nsteps; ++t) {
                // ======================= BACK =======================
                const int q = t - 4 - 3 * n;
                if (q >= 0 && q < Qb && (q & 1) == bw) {
                    const int sl = q & 1;
                    // stage n wrote ring n row q at step t - 1
                    const float4 X2 = sh.x2[n][sl][lane];
                    const float4 U0 = sh.u0[n][sl][lane];
                    const float4 U1 = sh.u1[n][sl][lane];
                    float4 Xo = X2;
                    if (!ALPHA1) {
                        const float4 YY = sh.y[q & (SP_YRING - 1)][lane];
                        Xo.x = (1.0f - a.alpha) * YY.x + a.alpha * X2.x;
                        Xo.y = (1.0f - a.alpha) * YY.y + a.alpha * X2.y;
                        Xo.z = (1.0f - a.alpha) * YY.z + a.alpha * X2.z;
                        Xo.w = (1.0f - a.alpha) * YY.w + a.alpha * X2.w;
                    }
                    float4 M4 = zero4, Q4 = zero4;
                    if (si.acc) {
                        float4 bm = zero4, bq = zero4;
                        if (need_prev) {
                            // DMA of row q was issued just before the previous row's stores
                            wait_vm_n(c1);
                            bm = sh.bst[bw][(q >> 1) & 1][0][lane];
                            bq = sh.bst[bw][(q >> 1) & 1][1][lane];
                        }
                        const float xs[CPL] = {Xo.x, Xo.y, Xo.z, Xo.w};
                        const float ms[CPL] = {bm.x, bm.y, bm.z, bm.w};
                        const float qs[CPL] = {bq.x, bq.y, bq.z, bq.w};
                        float m[CPL], qq[CPL];
#pragma unroll
                        for (int kk = 0; kk < CPL; ++kk) {
                            if (si.first) {
                                m[kk] = si.cb * xs[kk];
                                qq[kk] = si.cb * (xs[kk] * xs[kk]);
                            } else {
                                m[kk] = si.ca * ms[kk] + si.cb * xs[kk];
                                qq[kk] = si.ca * qs[kk] + si.cb * (xs[kk] * xs[kk]);
                            }
                        }
                        M4 = make_float4(m[0], m[1], m[2], m[3]);
                        Q4 = make_float4(qq[0], qq[1], qq[2], qq[3]);
                    }
                    // all LDS reads of this row (ring + staging) done before the staging
                    // buffer is re-targeted by the next DMA
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    const RowCursor rc = rc_cur;
                    cursor_advance(rm, rc_cur, 2);
                    if (q + 4 < Q) cursor_advance(rm, rc_dma, 2);
                    back_issue(q + 4, rc_dma);   // into the buffer just consumed (rows q, q + 4 share it)
                    asm volatile("" ::: "memory");
                    const bool rowcore = q >= qc0 && q < qc1;
                    {
                        const int ns = rowcore ? nst : 0;   // this row's stores (both steps)
                        c1 = c2 + 2 + ns;
                        c2 = ns;
                    }
                    // GEN: the lanes' columns of this row's segment
                    const SegGeo gr = seg_geo<GEN>(a, rc.p);
                    const int gjr = GEN ? gr.f0 + CPL * lane : gj0;
                    const bool corer = GEN ? (gjr < W && gjr >= gr.cc0 && gjr < gr.cc1) : core;
                    if (rowcore && corer) {
                        const size_t base = plane_off(gr.rp) + (size_t)rc.r * L + gjr;
                        st_nt(a.x[par_out] + base, Xo);
                        float* u2o = a.u2[par_out] + 2 * base;
                        st_nt(u2o, make_float4(U0.x, U1.x, U0.y, U1.y));
                        st_nt(u2o + 4, make_float4(U0.z, U1.z, U0.w, U1.w));
                        if (!ALPHA1) st_nt(a.x2[par_out] + base, X2);
                        // the accumulator / sample stores go out in the wave's next (idle) step
                        h_base = base; hM = M4; hQ = Q4; hX = Xo;
                    }
                    hold = rowcore;
                    if (GEN) hcore = corer;
                } else if (hold) {
                    flush_held();
                    hold = false;
                }
            step_barrier();
        }
        if (hold) flush_held();
    }

    // rel_err partial sums of this stream -> global, per segment's chain (deepinv's
    // early-stop test, per chain); the tracking stages wrote sh.red[segment][k - 1]
}

template <bool EXACT, bool ALPHA1, bool GEN>
__global__ void __launch_bounds__(TV_THREADS) tv_stream_kernel(const TvArgs a) {
    __shared__ StreamShared sh;
    __shared__ int s_stop[MAXG];
    __shared__ int s_flag, s_item, s_next;
    const int C = a.C;
    const long long step = (a.d_step ? *a.d_step : 0LL) + a.step_offset;
    const bool fresh = a.fresh_dev ? (*a.fresh_dev != 0) : (a.fresh_host != 0);
    {
        RowMap rm;
        build_rowmap(a, blockIdx.x, rm);
        stream_pass<EXACT, ALPHA1, GEN>(a, sh, rm, a.n_tv, true, step, fresh);
        if (!a.fin_inline) return;        // main-pass-only launch (kernel timing): no side effects
        // rel_err partial sums of this stream -> global, per segment's chain (deepinv's
        // early-stop test, per chain); the tracking stages wrote sh.red[segment][k - 1]
        lds_barrier();
        for (int tt = threadIdx.x; tt < SP_MAXSEG * SP_MAXST; tt += blockDim.x) {
            const int sg = tt / SP_MAXST, it = tt - sg * SP_MAXST;     // it = k - 1
            if (sg < rm.ns && it >= 2 && it <= a.n_tv - 2) {
                const int pl = rm.pl(sg) / a.st_nsegs;        // virtual plane -> plane
                const int g = a.per_chain_norm ? pl / C : 0;
                atomicAdd(&a.norms[((size_t)g * a.n_tv + it) * 2], (double)sh.red[sg][it][0]);
                atomicAdd(&a.norms[((size_t)g * a.n_tv + it) * 2 + 1], (double)sh.red[sg][it][1]);
            }
        }
    }
    // ---- step finalisation by the last workgroup to arrive (no second launch) ----
    // Every wave's stores and atomics complete, then one agent release per workgroup (writes the
    // XCD's dirty L2 lines back), then the arrival count.  The last
    // workgroup acquires before reading the rel-err sums or re-streaming a chain.
    wait_vm0();
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int old = __hip_atomic_fetch_add(a.arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_flag = (old == (int)gridDim.x - 1) ? 1 : 0;
        if (s_flag) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    wait_vm0();
    __syncthreads();
    if (!s_flag) return;
    // deepinv's early stop per chain: rel_err < tol at inner iteration t >= 2 -> the chain
    // stops after t + 1 iterations.  All (chain, t) tests in parallel: bit t of s_stop[g].
    const int G = a.B;
    for (int g = threadIdx.x; g < G; g += blockDim.x) s_stop[g] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < G * SP_MAXST; i += blockDim.x) {
        const int g = i / SP_MAXST, t = i - g * SP_MAXST;
        if (t >= 2 && t <= a.n_tv - 2) {
            const double nd = a.norms[((size_t)g * a.n_tv + t) * 2];
            const double nn = a.norms[((size_t)g * a.n_tv + t) * 2 + 1];
            const float rel = (float)sqrt(nd) / (float)sqrt(nn);
            if (rel < a.tol) atomicOr(&s_stop[g], 1 << t);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) { s_next = 0; s_item = 0; }
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
        const int m = s_stop[g];
        s_stop[g] = m ? (__ffs(m) - 1) + 1 : a.n_tv;
        if (m) s_item = 1;                    // some chain stopped early (benign race: all write 1)
    }
    __syncthreads();
    if (s_item == 0) s_next = 1 << 30;        // common case: nothing to redo, skip the scan
    // rare: re-stream every (plane, column segment) of a stopped chain alone with the stopped
    // iteration count (the step's inputs are intact: ping-pong state)
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            const int items = a.B * C * a.st_nsegs;
            int it = min(s_next, items), found = -1;
            for (; it < items; ++it)
                if (s_stop[(it / a.st_nsegs) / C] < a.n_tv) { found = it; break; }
            s_item = found;
            s_next = it + 1;
        }
        __syncthreads();
        const int item = __builtin_amdgcn_readfirstlane(s_item);
        if (item < 0) break;
        const int plane = item / a.st_nsegs;
        RowMap rm;
        plane_rowmap(a.H, item, rm);                 // the virtual plane (plane, column segment)
        const int nstop = __builtin_amdgcn_readfirstlane(s_stop[plane / C]);
        stream_pass<EXACT, ALPHA1, GEN>(a, sh, rm, nstop, false, step, fresh);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < a.B * a.n_tv * 2; i += blockDim.x) a.norms[i] = 0.0;
    if (threadIdx.x == 0) {
        *a.arrive = 0;
        if (a.fresh_dev) *a.fresh_dev = 0;
        if (a.advance_step && a.d_step) *a.d_step = *a.d_step + 1;   // (re-read: the start-of-kernel value measured +0.5 % here)
    }
}

// ---------------------------------------------------------------------------------------
// Small-batch fused step ("tile" variant, kernel_variant 4 / auto for small batches).
//
// Strong scaling gives each GPU 64/N chains: at 8 chains the row stream of a CU is ~24 core rows
// plus 2 x n_tv halo rows plus a 34-step pipeline fill, so the streaming pipeline spends most of
// a step filling and draining.  Here every (plane, band) tile is ONE workgroup and all tiles are
// resident at once: 16 waves x R rows x 256 columns (4 per lane) held in registers through all
// inner TV iterations (temporally blocked, n_tv halo rows recomputed by the neighbour bands, as
// the band kernel), with every load of the tile issued up front (the Philox / Box-Muller noise is
// computed while they fly; mean / sq LDS-DMA'd straight into LDS), 16-byte accumulator updates and
// the step finalised by the last workgroup (no second launch).  The per-element arithmetic is
// the stream kernel's in both modes (exact: bit-identical to the oracle; fast: bit-identical to
// the fast stream kernel).  Halos only at cuts inside a plane.  GEN: rows padded to a pitch ldw
// (W % 4 != 0) and / or column segments (W > 256) -- the stream kernel's segment geometry: tile =
// (plane, column segment, band), each segment's 256-column window carries n_tv halo columns at
// interior cuts.
// ---------------------------------------------------------------------------------------
// Core rows whose mean / sq rows a tile stages in LDS: all rows of the tile, at most 56 (112 KB; a 72-row tile
// of 8 waves x 9 rows has 52 core rows at n_tv = 10 -- tile_geometry keeps band_h within this)
constexpr int tile_mst_rows(int nw, int r) { return nw * r < 56 ? nw * r : 56; }

template <int R, int NW>
struct TileShared {
    float4 zrow[NW][WAVE];             // first-row z of each wave (read by the wave above)
    float4 urow[NW][WAVE];             // last-row u2[..., 0] of each wave (read by the wave below)
    float4 mst[tile_mst_rows(NW, R)][2][WAVE];   // mean / sq of the tile's core rows (LDS-DMA at the start)
    float2 red[MAXIT][NW][4];          // rel_err partial sums per (iteration, wave, 16-lane row of the wave)
    int s_stop[MAXG];
    int s_flag, s_item, s_next;
};

// before_u2: called by every wave once the tile's rel-err sums and X side are issued, before its u2 stores
// (the kernel's main pass: the step's arrival, so the u2 stores drain while the last workgroup finalises)
template <bool EXACT, bool ALPHA1, int R, bool GEN, int NW, typename BeforeU2>
__device__ __forceinline__ void sb_tile(const TvArgs& a, TileShared<R, NW>& sh, int plane, int seg, int band, int n_it,
                                        bool track, long long step, bool fresh, BeforeU2&& before_u2) {
    float x2[R][CPL], u0[R][CPL], u1[R][CPL];
    double* const nrm = a.norms;
    const int lane = threadIdx.x & (WAVE - 1);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int H = a.H, W = a.W, C = a.C, h = a.halo;
    const int L = GEN ? a.ldw : W;                     // row pitch
    const int b = plane / C, c = plane - b * C;
    const int r0 = band * a.band_h, r1 = min(H, r0 + a.band_h);
    const int e0 = max(0, r0 - h), e1 = min(H, r1 + h);
    // column window of the segment: core columns [cc0, cc1), wave window [f0, f0 + 256)
    const int cc0 = GEN ? seg * a.st_seg_w : 0;
    const int cc1 = GEN ? min(W, cc0 + a.st_seg_w) : W;
    const int f0 = GEN ? (max(0, cc0 - a.st_halo) & ~3) : 0;
    const int gj0 = f0 + CPL * lane;
    const int gjc = min(gj0, L - CPL);                 // DMA source column (every lane in bounds)
    const bool colok = gj0 < W;
    const bool corelane = GEN ? (colok && gj0 >= cc0 && gj0 < cc1) : colok;
    const int nreal = min(CPL, max(0, W - gj0));      // GEN: the lane's image (non-padding) columns
    const int lastk = W - 1 - gj0;                    // 0..3 on the lane holding column W-1
    const size_t HW = (size_t)H * L;
    const size_t E = (size_t)C * HW;
    const size_t BE = (size_t)a.B * E;
    const size_t poff = (size_t)plane * HW;
    const int par_in = (int)(step & 1), par_out = (int)((step + 1) & 1);
    const StepInfo si = step_info(a, step, a.mean[par_out]);
    const bool need_prev = si.acc && !si.first;
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);

    float z[R][CPL], yv[R][CPL];
    int gi[R];
    bool rv[R], core[R];
    // ---- 1. every load of the tile in flight: state and observation to registers, mean / sq by DMA
    float4 fX[R], fY[R], fU0[R], fU1[R], fXS[R];
    uint32_t fM[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        gi[r] = e0 + w * R + r;
        rv[r] = gi[r] < e1;
        core[r] = gi[r] >= r0 && gi[r] < r1;
        fX[r] = fY[r] = fU0[r] = fU1[r] = fXS[r] = zero4;
        fM[r] = 0u;
        if (rv[r] && colok) {
            const size_t base = poff + (size_t)gi[r] * L + gj0;
            fX[r] = ld4(a.x[par_in] + base);
            if (!fresh) {
                fU0[r] = ld4(a.u2[par_in] + 2 * base);
                fU1[r] = ld4(a.u2[par_in] + 2 * base + 4);
                if (!ALPHA1) fXS[r] = ld4(a.x2[par_in] + base);
            }
            fY[r] = ld4(a.yobs + (size_t)b * a.y_cs + (size_t)c * HW + (size_t)gi[r] * L + gj0);
            fM[r] = *reinterpret_cast<const uint32_t*>(a.mask + (size_t)b * a.m_cs + (size_t)gi[r] * L + gj0);
        }
    }
    if (need_prev && n_it >= 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (rv[r] && core[r]) {
                const size_t base = poff + (size_t)gi[r] * L + gjc;
                glds16(a.mean[par_in] + base, &sh.mst[gi[r] - r0][0][0]);
                glds16(a.sq[par_in] + base, &sh.mst[gi[r] - r0][1][0]);
            }
        }
    }
    // ---- 2. the noise of the tile's rows (no memory dependence: overlaps the loads)
    float Zn[R][CPL];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        // element index in the chain's unpadded C*H*W image: the noise does not depend on the row pitch
        const size_t e = ((size_t)c * H + (rv[r] ? gi[r] : 0)) * W + gj0;
        normal_quad(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step, TAG_LANGEVIN, (uint32_t)(e >> 2), Zn[r]);
        if (GEN) {
            const int esh = (int)(e & 3);               // the same for every lane of the row
            if (esh != 0) {                             // the lane's 4 elements span two quads
                float zq[CPL];
                normal_quad(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step, TAG_LANGEVIN, (uint32_t)(e >> 2) + 1u, zq);
                const float w8[8] = {Zn[r][0], Zn[r][1], Zn[r][2], Zn[r][3], zq[0], zq[1], zq[2], zq[3]};
#pragma unroll
                for (int i = 0; i < CPL; ++i)
                    Zn[r][i] = esh == 1 ? w8[i + 1] : (esh == 2 ? w8[i + 2] : w8[i + 3]);
            }
        }
    }
    // ---- 3. data term Y = (X + c1 g) + c2 Z, TV start state
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const bool ok = rv[r] && colok;
        const float X[CPL] = {fX[r].x, fX[r].y, fX[r].z, fX[r].w};
        const float yo[CPL] = {fY[r].x, fY[r].y, fY[r].z, fY[r].w};
        const float mk[CPL] = {(float)(fM[r] & 0xFFu), (float)((fM[r] >> 8) & 0xFFu), (float)((fM[r] >> 16) & 0xFFu),
                               (float)(fM[r] >> 24)};
        const float xs[CPL] = {fXS[r].x, fXS[r].y, fXS[r].z, fXS[r].w};
        const float us0[CPL] = {fU0[r].x, fU0[r].z, fU1[r].x, fU1[r].z};
        const float us1[CPL] = {fU0[r].y, fU0[r].w, fU1[r].y, fU1[r].w};
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            float Y;
            if (EXACT) {
                const float g = (-mk[k] * (X[k] - yo[k])) / a.sigma2;
                Y = (X[k] + a.c1 * g) + a.c2 * Zn[r][k];
            } else {
                const float g = (mk[k] * (yo[k] - X[k])) * a.inv_sigma2;
                Y = __builtin_fmaf(a.c2, Zn[r][k], __builtin_fmaf(a.c1, g, X[k]));
            }
            yv[r][k] = ok ? Y : 0.f;
            x2[r][k] = ok ? (fresh ? Y : (ALPHA1 ? X[k] : xs[k])) : 0.f;
            u0[r][k] = (ok && !fresh) ? us0[k] : 0.f;
            u1[r][k] = (ok && !fresh) ? us1[k] : 0.f;
            z[r][k] = 0.f;
        }
    }
    sh.urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
    __syncthreads();

    // ---- 4. inner TV iterations (deepinv 0.2.1 TVDenoiser, the stream kernel's arithmetic)
    const bool lastlane = gj0 + CPL == W;              // holds column W-1: no forward difference there
    // Trapezoid: the core rows need iteration j (1-based) only on rows [r0 - (n_it - j), r1 + (n_it - j))
    // for the dual and one row more below for the primal (the dual of a row reads the next row's z);
    // a wave none of whose rows is needed skips the phase (its stale rows feed only unneeded rows).
    const int wr0 = e0 + w * R, wr1 = wr0 + R;
    // The X side of the core rows' outputs (X, x2, accumulators / block means, sample) is final after the
    // last primal update.  48-row tiles issue it before the last dual update, so these stores drain while
    // it runs and only u2 waits for it (8 chains: 40.0 -> 38.8 us); the 32- and 72-row tiles measured
    // +2.3 % / +0.5 % that way and store after the last dual (profiles/r03s_tile_early_store_ab.txt)
    constexpr bool EARLY_X = R == 3;
    auto store_x_side = [&]() {
        if (need_prev) wait_vm0();                     // this wave's mean / sq DMA landed
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!(rv[r] && core[r] && corelane)) continue;
            const size_t base = poff + (size_t)gi[r] * L + gj0;
            float Xo[CPL];
#pragma unroll
            for (int k = 0; k < CPL; ++k)
                Xo[k] = ALPHA1 ? x2[r][k] : (1.0f - a.alpha) * yv[r][k] + a.alpha * x2[r][k];
            const float4 X4 = make_float4(Xo[0], Xo[1], Xo[2], Xo[3]);
            st_tile(a.x[par_out] + base, X4);
            if (!ALPHA1) st_tile(a.x2[par_out] + base, make_float4(x2[r][0], x2[r][1], x2[r][2], x2[r][3]));
            if (si.acc) {
                float4 bm = zero4, bq = zero4;
                if (need_prev) {
                    bm = sh.mst[gi[r] - r0][0][lane];
                    bq = sh.mst[gi[r] - r0][1][lane];
                }
                const float ms[CPL] = {bm.x, bm.y, bm.z, bm.w};
                const float qs[CPL] = {bq.x, bq.y, bq.z, bq.w};
                float m[CPL], q[CPL];
#pragma unroll
                for (int k = 0; k < CPL; ++k) {
                    if (si.first) {
                        m[k] = si.cb * Xo[k];
                        q[k] = si.cb * (Xo[k] * Xo[k]);
                    } else {
                        m[k] = si.ca * ms[k] + si.cb * Xo[k];
                        q[k] = si.ca * qs[k] + si.cb * (Xo[k] * Xo[k]);
                    }
                }
                const float4 M4 = make_float4(m[0], m[1], m[2], m[3]);
                const float4 Q4 = make_float4(q[0], q[1], q[2], q[3]);
                if (si.blockend) {
                    st_tile(a.blocks + (size_t)si.blk * BE + base, M4);
                    st_tile(a.blocks2 + (size_t)si.blk * BE + base, Q4);
                } else if (si.liveout) {
                    st_tile(a.mean[par_out] + base, M4);
                    st_tile(a.sq[par_out] + base, Q4);
                }
            }
            if (si.sample) st_tile(a.samples + (size_t)si.sidx * BE + base, X4);
        }
    };
    // one inner iteration; the last one (peeled: LAST is a compile-time constant at both call sites, so
    // the output addressing is not live across the loop) issues the X side between its two phases
    auto iteration = [&](const int it, auto last_tag) {
        constexpr bool LAST = decltype(last_tag)::value;
        const bool trk = track && it >= trk_lo(a) && it <= trk_hi(a);
        float sd = 0.f, sn = 0.f;
        const int span = n_it - 1 - it;
        const bool act_p = wr1 > r0 - span && wr0 < r1 + span + 1;
        const bool act_d = wr1 > r0 - span && wr0 < r1 + span;
        // primal: x = prox_tau_fx(x2 - tau nabla^T u2, Y); z = 2x - x2; x2 += rho (x - x2)
        const float4 up = (w > 0) ? sh.urow[w - 1][lane] : zero4;
        // the wave's first row -- the only one reading the hand-off from the wave above -- last, so that LDS
        // read's latency hides behind the other rows (-0.9 % at 8 chains, profiles/r03o_tile_row0_last_ab.txt)
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
            const int r = (rr + 1) % R;
            if (!act_p) break;
            const float u1l = __int_as_float(
                __builtin_amdgcn_update_dpp(0, __float_as_int(u1[r][CPL - 1]), 0x138 /* wave_shr:1 */, 0xF, 0xF, true));
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                // the row above: 0 above the tile's first row (the plane's top row or an artificial halo edge)
                const float pu = (r > 0) ? u0[r - 1][k] : f4get(up, k);
                const float u1left = (k > 0) ? u1[r][k - 1] : u1l;
                const float tt = ((pu - u0[r][k]) - u1[r][k]) + u1left;
                const float xo = x2[r][k];
                float xv, zv, xn;
                if (EXACT) {
                    xv = ((xo - a.tau * tt) + a.tau * yv[r][k]) / a.opt;
                    zv = 2.0f * xv - xo;
                    xn = xo + a.rho * (xv - xo);
                } else {
                    xv = __builtin_fmaf(a.tau, yv[r][k] - tt, xo) * a.inv_opt;
                    zv = __builtin_fmaf(2.0f, xv, -xo);
                    xn = __builtin_fmaf(a.rho, xv - xo, xo);
                }
                // rel-err terms of the counted rows (row-uniform test; lanes past W are masked once, at
                // the reduction: adding nothing and adding +0 leave a lane's sum identical)
                if (trk && core[r] && rv[r]) {
                    const bool real = !GEN || k < nreal;   // padding columns are not part of the norms
                    if (EXACT) {
                        const float d = real ? xo - xn : 0.f;
                        const float q = real ? xn + 1e-12f : 0.f;
                        sd = __builtin_fmaf(d, d, sd);
                        sn = __builtin_fmaf(q, q, sn);
                    } else {
                        const float d = real ? xv - xo : 0.f;
                        const float q = real ? xn : 0.f;
                        sd = __builtin_fmaf(d, d, sd);
                        sn = __builtin_fmaf(q, q, sn);
                    }
                }
                z[r][k] = zv;
                x2[r][k] = xn;
            }
        }
        if (act_p) sh.zrow[w][lane] = make_float4(z[0][0], z[0][1], z[0][2], z[0][3]);
        if (trk) {
            // 16-lane row sums by 4 DPP steps (no readlane round trip before the barrier); the 4 row sums of
            // each wave meet the other waves' at the end of the tile
            const float2 rs = row_sum2(corelane ? sd : 0.f, corelane ? sn : 0.f);
            if ((lane & 15) == 0) sh.red[it][w][lane >> 4] = rs;
        }
        __syncthreads();
        if (LAST && EARLY_X) store_x_side();
        // dual: u = prox_sigma_g_conj(u2 + sigma nabla z, ths); u2 += rho (u - u2)
        const float4 dn = (w < NW - 1) ? sh.zrow[w + 1][lane] : zero4;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!act_d) break;
            const float zr3 = __int_as_float(
                __builtin_amdgcn_update_dpp(0, __float_as_int(z[r][0]), 0x130 /* wave_shl:1 */, 0xF, 0xF, true));
            const bool down = gi[r] < H - 1;
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const float zc = z[r][k];
                const float zd = (r < R - 1) ? z[r + 1][k] : f4get(dn, k);
                const float zr = (k < CPL - 1) ? z[r][k + 1] : zr3;
                const float g0 = down ? (zd - zc) : 0.0f;
                float g1 = zr - zc;
                if (GEN) g1 = (lastk == k) ? 0.0f : g1;     // column W-1: no forward difference
                else if (k == CPL - 1) g1 = lastlane ? 0.0f : g1;
                const float uo0 = u0[r][k], uo1 = u1[r][k];
                if (EXACT) {
                    const float v0 = uo0 + a.sig_tv * g0;
                    const float v1 = uo1 + a.sig_tv * g1;
                    const float nrm = sqrtf(v0 * v0 + v1 * v1) / a.ths;
                    const float dd = fmaxf(nrm, 1.0f);
                    u0[r][k] = uo0 + a.rho * (v0 / dd - uo0);
                    u1[r][k] = uo1 + a.rho * (v1 / dd - uo1);
                } else {
                    const float v0 = __builtin_fmaf(a.sig_tv, g0, uo0);
                    const float v1 = __builtin_fmaf(a.sig_tv, g1, uo1);
                    const float s2 = __builtin_fmaf(v0, v0, v1 * v1);
                    const float f = fminf(1.0f, a.ths * __builtin_amdgcn_rsqf(s2));
                    u0[r][k] = __builtin_fmaf(a.rho, __builtin_fmaf(v0, f, -uo0), uo0);
                    u1[r][k] = __builtin_fmaf(a.rho, __builtin_fmaf(v1, f, -uo1), uo1);
                }
            }
        }
        if (act_d) sh.urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
        __syncthreads();
    };
    for (int it = 0; it < n_it - 1; ++it) iteration(it, std::false_type{});
    if (n_it > 0) iteration(n_it - 1, std::true_type{});
    // ---- 5. rel_err partial sums -> the chain's norms (one fp64 atomic per iteration and workgroup)
    if (track) {
        const int t = threadIdx.x;
        if (t >= trk_lo(a) && t <= trk_hi(a) && t < n_it) {
            double sd = 0.0, sn = 0.0;
            for (int ww = 0; ww < NW; ++ww)
                for (int q = 0; q < 4; ++q) { sd += sh.red[t][ww][q].x; sn += sh.red[t][ww][q].y; }
            if (!EXACT) sd *= (double)(a.rho * a.rho);     // fast sums hold (x - x2_prev)^2
            // workgroup x adds to copy x % norm_copies (x & 7 = its XCD when there are 8): fewer adds queue
            // on one address when many tiles share a chain
            double* const nc = nrm + (size_t)(blockIdx.x % a.norm_copies) * ((size_t)a.B * a.n_tv * 2);
            atomicAdd(&nc[((size_t)b * a.n_tv + t) * 2], sd);
            atomicAdd(&nc[((size_t)b * a.n_tv + t) * 2 + 1], sn);
        }
    }
    // ---- 6. the core rows out: the X side (48-row tiles: issued before the last dual update), u2
    if (!EARLY_X || n_it <= 0) store_x_side();
    before_u2();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!(rv[r] && core[r] && corelane)) continue;
        const size_t base = poff + (size_t)gi[r] * L + gj0;
        float* u2o = a.u2[par_out] + 2 * base;
        st_tile(u2o, make_float4(u0[r][0], u1[r][0], u0[r][1], u1[r][1]));
        st_tile(u2o + 4, make_float4(u0[r][2], u1[r][2], u0[r][3], u1[r][3]));
    }
}

template <bool EXACT, bool ALPHA1, int R, bool GEN, int NW>
__global__ void __launch_bounds__(NW * WAVE) tv_tile_kernel(const TvArgs a) {
    __shared__ TileShared<R, NW> sh;
    constexpr bool SPLIT = NW == 8;                    // two-phase arrival (below)
    const long long step = (a.d_step ? *a.d_step : 0LL) + a.step_offset;
    const bool fresh = a.fresh_dev ? (*a.fresh_dev != 0) : (a.fresh_host != 0);
    const int P = a.B * a.C;
    const int T = a.nbands * (GEN ? a.st_nsegs : 1);  // tiles per plane: (column segment, band)
    {
        // the P * T tiles, plane-major, cut into 8 equal runs, one per XCD (blocks x and x + 8 share one):
        // the tiles of a plane share an XCD's L2 for their halo rows, and every XCD gets work even when
        // there are fewer than 8 planes (one image at the CLI's batch 1)
        const int N = P * T, per = (N + 7) / 8;
        const int x = blockIdx.x, xcd = x & 7, k = x >> 3;
        const int item = xcd * per + k;
        // Arrival.  The 72-row tiles (SPLIT) arrive before their u2 stores, so those drain while the last
        // workgroup finalises (16 chains 68.3 -> 67.0 us; the 16-wave tiles measured +1-1.4 % that way,
        // profiles/r03s_tile_two_phase_ab.txt): the counter a.arrive then holds two counts, the low 16 bits
        // the workgroups whose rel-err sums and X side are complete (phase 1: the last one finalises the
        // step), the high bits those whose u2 stores are complete too (phase 2: the rare early-stop recompute
        // rewrites outputs, so it waits for them); the last workgroup takes both counts out at the end, by
        // one atomic add.  The other tiles arrive once everything is stored (phase 1 only).
        auto arrive = [&]() {
            if (!a.fin_inline) return;
            wait_vm0();
            __syncthreads();
            if (threadIdx.x == 0) {
        // Without fences: every output of this kernel is an sc1 (write-through) store and every rel-err sum
        // an agent-scope atomic; each wave waited vmcnt(0) before the barrier above, one lane per workgroup
        // adds to the arrival counter, and the workgroup whose add returns the last count reads the sums by
        // agent atomics (MI355X_MICROARCH.md: "8-B agent atomics both sides" with its hand-off row 1; a
        // release + acquire pair cost 1.1 us per step here).  Nothing else this launch wrote is read by it
        // (the rare redo reads the step's inputs, written by the previous launch).
                const int old = __hip_atomic_fetch_add(a.arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                sh.s_flag = ((old & 0xFFFF) == (int)gridDim.x - 1) ? 1 : 0;
            }
            wait_vm0();
            __syncthreads();
        };
        if (item < N) {
            const int plane = item / T, t = item - plane * T;
            const int seg = GEN ? t / a.nbands : 0;
            const int band = t - seg * a.nbands;
            if constexpr (SPLIT) sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, a.n_tv, true, step, fresh, arrive);
            else sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, a.n_tv, true, step, fresh, [] {});
        }
        if (!SPLIT || item >= N) arrive();
    }
    if (!a.fin_inline) return;
    if (!sh.s_flag) {
        if (!SPLIT) return;
        // phase 2: this workgroup's u2 stores are complete
        wait_vm0();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(a.arrive, 1 << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    // ---- step finalisation by the last workgroup to arrive (as tv_stream_kernel) ----
    const int G = a.B;
    for (int g = threadIdx.x; g < G; g += blockDim.x) sh.s_stop[g] = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < G * MAXIT; i += blockDim.x) {
        const int g = i / MAXIT, t = i - g * MAXIT;
        if (t >= trk_lo(a) && t <= trk_hi(a) && t < a.n_tv) {
            // read by agent-scope atomics (+0.0, returning), as they were written: 8-B agent atomics on both
            // sides of the hand-off, performed where the producers' adds were
            double nd = 0.0, nn = 0.0;
            for (int cp = 0; cp < a.norm_copies; ++cp) {   // the copies in a fixed order
                double* const nc = a.norms + (size_t)cp * ((size_t)a.B * a.n_tv * 2);
                nd += __hip_atomic_fetch_add(&nc[((size_t)g * a.n_tv + t) * 2], 0.0, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
                nn += __hip_atomic_fetch_add(&nc[((size_t)g * a.n_tv + t) * 2 + 1], 0.0, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
            }
            const float rel = (float)sqrt(nd) / (float)sqrt(nn);
            if (rel < a.tol) atomicOr(&sh.s_stop[g], 1 << t);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) sh.s_item = 0;
    __syncthreads();
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
        const int m = sh.s_stop[g];
        sh.s_stop[g] = m ? (__ffs(m) - 1) + 1 : a.n_tv;
        if (m) sh.s_item = 1;
    }
    __syncthreads();
    if (sh.s_item) {
        // rare: redo every tile of a stopped chain with the stopped iteration count (inputs intact), once every
        // other workgroup's stores are complete (phase 2; all of them have arrived, so each will count: bounded
        // wait only as a guard)
        if (SPLIT && threadIdx.x == 0) {
            for (int spin = 0; spin < (1 << 24); ++spin) {
                if ((__hip_atomic_load(a.arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 16) >= (int)gridDim.x - 1) break;
                __builtin_amdgcn_s_sleep(2);
            }
        }
        wait_vm0();
        __syncthreads();
        for (int item = 0; item < P * T; ++item) {
            const int plane = item / T, t = item - plane * T;
            const int seg = GEN ? t / a.nbands : 0;
            const int band = t - seg * a.nbands;
            const int nstop = __builtin_amdgcn_readfirstlane(sh.s_stop[plane / a.C]);
            if (nstop < a.n_tv) {
                sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, nstop, false, step, fresh, [] {});
                wait_vm0();
                __syncthreads();
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < a.B * a.n_tv * 2 * a.norm_copies; i += blockDim.x) a.norms[i] = 0.0;
    if (threadIdx.x == 0) {
        // both counts out (the other workgroups' phase-2 adds may still be landing: an add, not a store); the
        // counter is 0 once the kernel has completed
        const int G1 = (int)gridDim.x;
        if (SPLIT) __hip_atomic_fetch_add(a.arrive, -(G1 + ((G1 - 1) << 16)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *a.arrive = 0;
        if (a.fresh_dev) *a.fresh_dev = 0;
        if (a.advance_step && a.d_step) *a.d_step = step - a.step_offset + 1;   // the value read at the start: no dependent load
    }
}

// ---------------------------------------------------------------------------------------
// Generic elementwise kernels (opaque closures; also the first / last steps of fused paths)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ long long read_step(const long long* d, long long off) {
    return (d ? *d : 0LL) + off;
}

__global__ void normal_fill_kernel(float* out, int B, long long E, unsigned long long seed, int chain0,
                                   const long long* d_step, long long off, uint32_t tag) {
    const long long step = read_step(d_step, off);
    const long long Q = (E + 3) >> 2;
    const long long total = (long long)B * Q;
    for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int b = (int)(t / Q);
        const long long q = t - (long long)b * Q;
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)step, tag, (uint32_t)q, z);
        const long long e = q << 2;
        float* o = out + (size_t)b * E + e;
        if (e + 3 < E && ((E & 3) == 0)) {
            *reinterpret_cast<float4*>(o) = make_float4(z[0], z[1], z[2], z[3]);
        } else {
            for (int j = 0; j < 4; ++j)
                if (e + j < E) o[j] = z[j];
        }
    }
}

// Y = (X + c1 g) + c2 Z   (restoration_algorithms.py:236)
__global__ void langevin_update_kernel(const float* X, const float* g, float* Y, int B, long long E,
                                       float c1, float c2, unsigned long long seed, int chain0,
                                       const long long* d_step, long long off) {
    // grid: (quads of a chain, chain); one noise quad = 4 consecutive elements of the chain
    const long long step = read_step(d_step, off);
    const long long Q = (E + 3) >> 2;
    const int b = blockIdx.y;
    const bool vec = (E & 3) == 0;
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < Q;
         q += (long long)gridDim.x * blockDim.x) {
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)step, TAG_LANGEVIN, (uint32_t)q, z);
        const size_t i0 = (size_t)b * E + (size_t)(q << 2);
        if (vec) {
            const float4 x = ld4(X + i0), gg = ld4(g + i0);
            st4(Y + i0, (x.x + c1 * gg.x) + c2 * z[0], (x.y + c1 * gg.y) + c2 * z[1],
                (x.z + c1 * gg.z) + c2 * z[2], (x.w + c1 * gg.w) + c2 * z[3]);
        } else {
            for (int j = 0; j < 4; ++j)
                if ((q << 2) + j < E) Y[i0 + j] = (X[i0 + j] + c1 * g[i0 + j]) + c2 * z[j];
        }
    }
}


// ---------------------------------------------------------------------------------------
// Deblurring data term (sampling_images.py:304-341): g = -A^T(A x - y) / sigma2 with
// A x = conv2d(pad(x, l, circular), hconv) and A^T r = conv2d(pad(r, l, circular), hcorr),
// depthwise, K = 2l+1 taps per side (the same for every channel).  One workgroup per 64 x 64
// output tile of a plane: x is staged in LDS with a 2l halo (circular wrap on load, 16-byte loads
// where the tile does not wrap), r = A x - y is formed in LDS on the tile + l halo, then
// g = -(A^T r) / sigma2.  Register blocking over rows AND columns: a thread produces a 4-column x
// M-row block, reading each of its M + 2l input rows once (ceil((4 + 2l) / 4) ds_read_b128) and
// adding that row into every output row it touches -- LDS traffic per output falls from
// K x (4 + 2l) floats / 4 to (M + 2l) x (4 + 2l) / (4 M), so the 2 x K^2 multiply-adds (VALU), not
// LDS, bound the kernel.  Every output's sum still runs over (u, v) in increasing order (the same
// arithmetic as a plain per-output loop; `oracle.blur_grad_tap_order` pins it bit for bit in exact
// mode).  The taps are kernel arguments (compile-time indices -> SGPR operands).
// With Y != NULL the Langevin update Y = (X + c1 g) + c2 Z is fused (g is never stored; X is read
// from the staged tile).
// ---------------------------------------------------------------------------------------
constexpr int BL_TH = 64, BL_TW = 64, BL_MAXL = 8, BL_THREADS = 256;
constexpr int BL_MAXK = 2 * BL_MAXL + 1;
constexpr int BL_MG = 4;                          // output rows per thread in the A^T r pass (16 x 16 blocks)

// rows per thread of the r = A x - y pass: the smallest M >= 4 whose blocks fit one pass of the workgroup
__host__ __device__ constexpr int bl_mr(int L) {
    int m = 4;
    while (m < 16 && ((BL_TW + 2 * L + 3) / 4) * ((BL_TH + 2 * L + m - 1) / m) > BL_THREADS) ++m;
    return m;
}

struct BlurArgs {
    const float* X;
    const float* y;
    long long y_cs;
    float hconv[BL_MAXK * BL_MAXK];
    float hcorr[BL_MAXK * BL_MAXK];
    float sconv_r[BL_MAXK], sconv_c[BL_MAXK];      // rank-1 factors (separable fast path): h[u][v] = r[u] c[v]
    float scorr_r[BL_MAXK], scorr_c[BL_MAXK];
    float* g;
    float* Y;
    int B, C, H, W;
    float sigma2, inv_sigma2, c1, c2;
    unsigned long long seed;
    int chain0;
    const long long* d_step;
    long long off;
    int tiles_x, tiles_y;
};

// acc[m][0..3] += sum_v h[u][v] * row[k + v] for every output row m that input row `ir` feeds (u = ir - m)
template <bool EXACT, int K, int M, int SEG>
__device__ __forceinline__ void bl_row_accumulate(const float* __restrict__ h, const float (&row)[SEG * 4], int ir,
                                                  float (&acc)[M][4]) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int u = ir - m;
        if (u < 0 || u >= K) continue;                 // compile-time after unrolling
#pragma unroll
        for (int v = 0; v < K; ++v) {
            const float hv = h[u * K + v];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                acc[m][k] = EXACT ? acc[m][k] + hv * row[k + v] : __builtin_fmaf(hv, row[k + v], acc[m][k]);
        }
    }
}


template <int SEG>
__device__ __forceinline__ void bl_load_row(const float* p, float (&row)[SEG * 4]) {
#pragma unroll
    for (int sg = 0; sg < SEG; ++sg) {
        const float4 v = *reinterpret_cast<const float4*>(p + 4 * sg);
        row[4 * sg] = v.x; row[4 * sg + 1] = v.y; row[4 * sg + 2] = v.z; row[4 * sg + 3] = v.w;
    }
}

// One workgroup per (plane, tile), 1-D grid; three resident per CU for l <= 4 (168 VGPRs, 47 KB of LDS).
// (A persistent variant that DMA'd the next tile into a second buffer during the passes measured slower:
// two workgroups per CU hide less than three)
#ifndef PSGLA_BLUR_WPE
#define PSGLA_BLUR_WPE 3
#endif
template <bool EXACT, int L>
__global__ void __launch_bounds__(BL_THREADS, (L <= 4 ? PSGLA_BLUR_WPE : 1)) blur_grad_kernel(const BlurArgs a) {
    constexpr int K = 2 * L + 1;
    constexpr int MR = bl_mr(L);
    constexpr int RQ = (BL_TW + 2 * L + 3) / 4, RB = (BL_TH + 2 * L + MR - 1) / MR;   // r pass: strips x row blocks
    constexpr int XH = BL_TH + 4 * L, XW = BL_TW + 4 * L, XQ = XW / 4;                 // staged x (XW % 4 == 0)
    constexpr int XHA = RB * MR + 2 * L;              // rows the r pass may read (last block: rows past RH unused)
    constexpr int RHA = RB * MR;
    // x rows unpadded (XS == XW: the staged tile is one contiguous array, so LDS-DMA rows land back to
    // back); + 8 floats: the last strip's row segment may run up to 6 floats past the last row
    constexpr int XS = XW, RS = ((BL_TW + 2 * L + 3) & ~3) + 4;
    constexpr int SEG = (4 + 2 * L + 3) / 4;                                        // float4 reads per row segment
    constexpr int TQ = BL_TW / 4, TB = BL_TH / BL_MG;
    constexpr int NXI = (XH * XQ + BL_THREADS - 1) / BL_THREADS;                     // staging chunks per thread
    static_assert(TQ * TB == BL_THREADS, "A^T r pass: one block per thread");
    __shared__ __attribute__((aligned(16))) float xs[XHA * XS + 8];
    __shared__ __attribute__((aligned(16))) float rs[RHA * RS];
    const int H = a.H, W = a.W;
    const size_t HW = (size_t)H * W;
    const bool vec = (W & 3) == 0;
    const bool dma = (L & 1) == 0 && vec;   // even l on a 4-aligned width: every staging chunk is one aligned 16-B run
    const int per_plane = a.tiles_x * a.tiles_y;
    const long long step = (a.d_step ? *a.d_step : 0LL) + a.off;
    // circular index without loops: one correction covers every offset an output uses when 2l <= n; tiny
    // planes (and the unused rows past a partial tile) take the exact modulo
    auto wrap = [](int v, int n) {
        if ((unsigned)v < (unsigned)n) return v;
        const int r = v + (v < 0 ? n : -n);
        if ((unsigned)r < (unsigned)n) return r;
        const int m = v % n;
        return m < 0 ? m + n : m;
    };
    struct Tile { int plane, b, c, i0, j0; };
    auto tile_of = [&](int id) {
        Tile tl;
        tl.plane = id / per_plane;
        const int r = id - tl.plane * per_plane, ty = r / a.tiles_x, tx = r - ty * a.tiles_x;
        tl.b = tl.plane / a.C; tl.c = tl.plane - tl.b * a.C;
        tl.i0 = ty * BL_TH; tl.j0 = tx * BL_TW;
        return tl;
    };
    const int t = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    // r pass geometry: 4-column x MR-row blocks of rows i0-l .. i0+TH+l-1, cols j0-l .. j0+TW+l-1
    const bool rblk = t < RQ * RB;
    const int rq = t % RQ, rb = t / RQ;
    const int q = 4 * rq, p0 = rb * MR;
    float yv[MR][4];
    // the observation under this thread's r block (registers)
    auto load_y = [&](const Tile& tl) {
        if (!rblk) return;
        const float* yp = a.y + (size_t)tl.b * a.y_cs + (size_t)tl.c * HW;
        const int gj = tl.j0 - L + q;
        const bool yvec = (L & 3) == 0 && vec && gj >= 0 && gj + 3 < W;
#pragma unroll
        for (int m = 0; m < MR; ++m) {
            yv[m][0] = yv[m][1] = yv[m][2] = yv[m][3] = 0.f;
            if (p0 + m < BL_TH + 2 * L) {
                const float* yrow = yp + (size_t)wrap(tl.i0 - L + p0 + m, H) * W;
                if (yvec) {
                    const float4 v = ld4(yrow + gj);
                    yv[m][0] = v.x; yv[m][1] = v.y; yv[m][2] = v.z; yv[m][3] = v.w;
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (q + k < BL_TW + 2 * L) yv[m][k] = yrow[wrap(gj + k, W)];
                }
            }
        }
    };
    // x on rows i0-2l .. i0+TH+2l-1, cols j0-2l .. j0+TW+2l-1 (circular padding applied twice), in
    // 4-column chunks: chunk n of the tile -> buf[4n].  LDS-DMA (no registers, all in flight at once) or,
    // for odd l / widths not a multiple of 4, element loads through registers.
    auto stage_x = [&](const Tile& tl, float* buf) {
        const float* xp = a.X + (size_t)tl.plane * HW;
        if (dma) {
#pragma unroll
            for (int it = 0; it < NXI; ++it) {
                const int n = it * BL_THREADS + t;
                if (n < XH * XQ) {
                    const int p = n / XQ, qq = n - p * XQ;
                    glds16(xp + (size_t)wrap(tl.i0 - 2 * L + p, H) * W + wrap(tl.j0 - 2 * L + 4 * qq, W),
                           &buf[4 * (it * BL_THREADS + 64 * wv)]);
                }
            }
            return;
        }
        for (int n = t; n < XH * XQ; n += BL_THREADS) {
            const int p = n / XQ, qq = n - p * XQ;
            const float* rowp = xp + (size_t)wrap(tl.i0 - 2 * L + p, H) * W;
            const int gj = tl.j0 - 2 * L + 4 * qq;
            float4 v;
            v.x = rowp[wrap(gj, W)]; v.y = rowp[wrap(gj + 1, W)];
            v.z = rowp[wrap(gj + 2, W)]; v.w = rowp[wrap(gj + 3, W)];
            *reinterpret_cast<float4*>(&buf[4 * n]) = v;
        }
    };

    // workgroups are dealt round-robin to the 8 XCDs: give each XCD a contiguous run of tiles so the
    // halo rows / columns a tile shares with its neighbours are re-read from the same L2 (-5 %; the
    // loads-and-stores floor 44 -> 31 us)
    int tid;
    {
        const int ntiles = per_plane * a.B * a.C, bid = blockIdx.x;
        const int xcd = bid & 7, k = bid >> 3, qt = ntiles >> 3, rt = ntiles & 7;
        tid = xcd * qt + min(xcd, rt) + k;
    }
    const Tile tl = tile_of(tid);
    load_y(tl);                              // y first: it has landed by the time the tile has
    stage_x(tl, xs);
    wait_vm0();                              // this wave's x chunks and y landed
    __syncthreads();
    {
        const float* xb = xs;
        // r = A x - y
        if (rblk) {
            float acc[MR][4];
#pragma unroll
            for (int m = 0; m < MR; ++m) acc[m][0] = acc[m][1] = acc[m][2] = acc[m][3] = 0.f;
#pragma unroll
            for (int ir = 0; ir < MR + 2 * L; ++ir) {
                float row[SEG * 4];
                bl_load_row<SEG>(&xb[(p0 + ir) * XS + q], row);
                bl_row_accumulate<EXACT, K, MR, SEG>(a.hconv, row, ir, acc);
            }
#pragma unroll
            for (int m = 0; m < MR; ++m)
                *reinterpret_cast<float4*>(&rs[(p0 + m) * RS + q]) =
                    make_float4(acc[m][0] - yv[m][0], acc[m][1] - yv[m][1], acc[m][2] - yv[m][2], acc[m][3] - yv[m][3]);
        }
        __syncthreads();
        // g = -(A^T r) / sigma2 on the tile (+ the fused Langevin update): 4-column x 4-row blocks
        const int gq = 4 * (t % TQ), gp0 = BL_MG * (t / TQ);
        const int j = tl.j0 + gq;
        if (j < W && tl.i0 + gp0 < H) {
            float acc[BL_MG][4];
#pragma unroll
            for (int m = 0; m < BL_MG; ++m) acc[m][0] = acc[m][1] = acc[m][2] = acc[m][3] = 0.f;
#pragma unroll
            for (int ir = 0; ir < BL_MG + 2 * L; ++ir) {
                float row[SEG * 4];
                bl_load_row<SEG>(&rs[(gp0 + ir) * RS + gq], row);
                bl_row_accumulate<EXACT, K, BL_MG, SEG>(a.hcorr, row, ir, acc);
            }
#pragma unroll
            for (int m = 0; m < BL_MG; ++m) {
                const int i = tl.i0 + gp0 + m;
                if (i >= H) break;
                float gv[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) gv[kk] = EXACT ? (-acc[m][kk]) / a.sigma2 : (-acc[m][kk]) * a.inv_sigma2;
                const size_t e0 = (size_t)tl.c * HW + (size_t)i * W + j;   // element index within the chain
                const size_t o = (size_t)tl.b * a.C * HW + e0;
                if (a.Y) {
                    float z[4];
                    if (vec) {
                        normal_quad(a.seed, (uint32_t)(a.chain0 + tl.b), (uint32_t)step, TAG_LANGEVIN, (uint32_t)(e0 >> 2), z);
                    } else {
#pragma unroll
                        for (int kk = 0; kk < 4; ++kk)
                            z[kk] = normal_elem(a.seed, (uint32_t)(a.chain0 + tl.b), (uint32_t)step, TAG_LANGEVIN,
                                                (uint64_t)(e0 + kk));
                    }
                    // X of the tile from the staged copy (the same values as a.X)
                    const float* xr = &xb[(gp0 + m + 2 * L) * XS + gq + 2 * L];
                    float yo[4];
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) yo[kk] = (xr[kk] + a.c1 * gv[kk]) + a.c2 * z[kk];
                    if (vec) {
                        *reinterpret_cast<float4*>(a.Y + o) = make_float4(yo[0], yo[1], yo[2], yo[3]);
                    } else {
#pragma unroll
                        for (int kk = 0; kk < 4; ++kk)
                            if (j + kk < W) a.Y[o + kk] = yo[kk];
                    }
                } else if (vec) {
                    *reinterpret_cast<float4*>(a.g + o) = make_float4(gv[0], gv[1], gv[2], gv[3]);
                } else {
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
                        if (j + kk < W) a.g[o + kk] = gv[kk];
                }
            }
        }
    }
}

// Separable fast path.  The reference's blur kernels are rank 1 (h_ = h^T h, sampling_images.py:306-313), so
// in fast mode (the tolerance contract) each (2l+1)^2 stencil runs as a row pass and a column pass:
// 2 (2l+1) instead of (2l+1)^2 multiply-adds per output and pass.  Four passes through two LDS buffers:
//   x (LDS-DMA, as the 2-D kernel) -> hx = rows(x) -> r = cols(hx) - y (over x's buffer) -> hr = rows(r)
//   (over hx's buffer) -> g = cols(hr), fused Langevin update with X re-read from HBM.
// Chosen on the host only when the taps factor to fp32 rounding (psgla_blur_grad); exact mode keeps the 2-D
// kernel and its tap order.
template <int L>
__global__ void __launch_bounds__(BL_THREADS, (L <= 4 ? 3 : 1)) blur_sep_kernel(const BlurArgs a) {
    constexpr int K = 2 * L + 1;
    constexpr int MR = bl_mr(L);
    constexpr int RQ = (BL_TW + 2 * L + 3) / 4, RB = (BL_TH + 2 * L + MR - 1) / MR;   // r blocks (cols pass 1)
    constexpr int XH = BL_TH + 4 * L, XW = BL_TW + 4 * L, XQ = XW / 4;
    constexpr int XHA = RB * MR + 2 * L;
    constexpr int XS = XW;                                        // staged x: contiguous rows (LDS-DMA)
    constexpr int RS = ((BL_TW + 2 * L + 3) & ~3) + 4;             // r rows (in x's buffer)
    constexpr int HS = ((BL_TW + 2 * L + 3) & ~3) + 4;             // hx / hr rows
    constexpr int SEG = (4 + 2 * L + 3) / 4;
    constexpr int NXI = (XH * XQ + BL_THREADS - 1) / BL_THREADS;
    constexpr int TQ = BL_TW / 4, TB = BL_TH / BL_MG;
    // rows pass 1 (hx on all XHA rows, RQ strips) and rows pass 2 (hr on RB*MR rows, TQ strips): rows per thread
    constexpr int M1 = (XHA * RQ + BL_THREADS - 1) / BL_THREADS;   // rows per strip block, pass 1
    constexpr int B1 = (XHA + M1 - 1) / M1;
    constexpr int M2 = (RB * MR * TQ + BL_THREADS - 1) / BL_THREADS;
    constexpr int B2 = (RB * MR + M2 - 1) / M2;
    static_assert(TQ * TB == BL_THREADS, "cols pass 2: one block per thread");
    constexpr int ABUF = (XHA * XS + 8 > RB * MR * RS) ? XHA * XS + 8 : RB * MR * RS;
    constexpr int BBUF = (B1 * M1 > RB * MR ? B1 * M1 : RB * MR) * HS;
    __shared__ __attribute__((aligned(16))) float bufA[ABUF];
    __shared__ __attribute__((aligned(16))) float bufB[BBUF];
    const int H = a.H, W = a.W;
    const size_t HW = (size_t)H * W;
    const bool vec = (W & 3) == 0;
    const bool dma = (L & 1) == 0 && vec;
    const int per_plane = a.tiles_x * a.tiles_y;
    const long long step = (a.d_step ? *a.d_step : 0LL) + a.off;
    auto wrap = [](int v, int n) {
        if ((unsigned)v < (unsigned)n) return v;
        const int r = v + (v < 0 ? n : -n);
        if ((unsigned)r < (unsigned)n) return r;
        const int m = v % n;
        return m < 0 ? m + n : m;
    };
    int tid;
    {
        const int ntiles = per_plane * a.B * a.C, bid = blockIdx.x;
        const int xcd = bid & 7, k = bid >> 3, qt = ntiles >> 3, rt = ntiles & 7;
        tid = xcd * qt + min(xcd, rt) + k;
    }
    const int plane = tid / per_plane;
    const int rem = tid - plane * per_plane, ty = rem / a.tiles_x, tx = rem - ty * a.tiles_x;
    const int b = plane / a.C, c = plane - b * a.C;
    const int i0 = ty * BL_TH, j0 = tx * BL_TW;
    const float* xp = a.X + (size_t)plane * HW;
    const float* yp = a.y + (size_t)b * a.y_cs + (size_t)c * HW;
    const int t = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    // r blocks (cols pass 1): 4 columns x MR rows; y under the block first
    const bool rblk = t < RQ * RB;
    const int rq = t % RQ, rb = t / RQ;
    const int q = 4 * rq, p0 = rb * MR;
    float yv[MR][4];
    if (rblk) {
        const int gj = j0 - L + q;
        const bool yvec = (L & 3) == 0 && vec && gj >= 0 && gj + 3 < W;
#pragma unroll
        for (int m = 0; m < MR; ++m) {
            yv[m][0] = yv[m][1] = yv[m][2] = yv[m][3] = 0.f;
            if (p0 + m < BL_TH + 2 * L) {
                const float* yrow = yp + (size_t)wrap(i0 - L + p0 + m, H) * W;
                if (yvec) {
                    const float4 v = ld4(yrow + gj);
                    yv[m][0] = v.x; yv[m][1] = v.y; yv[m][2] = v.z; yv[m][3] = v.w;
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (q + k < BL_TW + 2 * L) yv[m][k] = yrow[wrap(gj + k, W)];
                }
            }
        }
    }
    if (dma) {
#pragma unroll
        for (int it = 0; it < NXI; ++it) {
            const int n = it * BL_THREADS + t;
            if (n < XH * XQ) {
                const int p = n / XQ, qq = n - p * XQ;
                glds16(xp + (size_t)wrap(i0 - 2 * L + p, H) * W + wrap(j0 - 2 * L + 4 * qq, W),
                       &bufA[4 * (it * BL_THREADS + 64 * wv)]);
            }
        }
    } else {
        for (int n = t; n < XH * XQ; n += BL_THREADS) {
            const int p = n / XQ, qq = n - p * XQ;
            const float* rowp = xp + (size_t)wrap(i0 - 2 * L + p, H) * W;
            const int gj = j0 - 2 * L + 4 * qq;
            float4 v;
            v.x = rowp[wrap(gj, W)]; v.y = rowp[wrap(gj + 1, W)];
            v.z = rowp[wrap(gj + 2, W)]; v.w = rowp[wrap(gj + 3, W)];
            *reinterpret_cast<float4*>(&bufA[4 * n]) = v;
        }
    }
    wait_vm0();
    __syncthreads();
    // rows pass 1: hx[p][q] = sum_v c[v] x[p][q + v], p < XHA (rows past XH: unused), q < 4 RQ
    if (t < RQ * B1) {
        const int sq = 4 * (t % RQ), sp = M1 * (t / RQ);
#pragma unroll
        for (int m = 0; m < M1; ++m) {
            if (sp + m >= XHA) break;
            float row[SEG * 4];
            bl_load_row<SEG>(&bufA[(sp + m) * XS + sq], row);
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int v = 0; v < K; ++v)
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] = __builtin_fmaf(a.sconv_c[v], row[k + v], acc[k]);
            *reinterpret_cast<float4*>(&bufB[(sp + m) * HS + sq]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
    }
    __syncthreads();
    // cols pass 1: r[p][q] = sum_u r_[u] hx[p + u][q] - y  (into x's buffer: x is dead)
    float racc[MR][4];
#pragma unroll
    for (int m = 0; m < MR; ++m) racc[m][0] = racc[m][1] = racc[m][2] = racc[m][3] = 0.f;
    if (rblk) {
        float (&acc)[MR][4] = racc;
#pragma unroll
        for (int ir = 0; ir < MR + 2 * L; ++ir) {
            const float4 v4 = *reinterpret_cast<const float4*>(&bufB[(p0 + ir) * HS + q]);
            const float hv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int m = 0; m < MR; ++m) {
                const int u = ir - m;
                if (u < 0 || u >= K) continue;
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[m][k] = __builtin_fmaf(a.sconv_r[u], hv[k], acc[m][k]);
            }
        }
    }
    __syncthreads();                                       // (x's buffer was last read by rows pass 1)
    if (rblk) {
#pragma unroll
        for (int m = 0; m < MR; ++m)
            *reinterpret_cast<float4*>(&bufA[(p0 + m) * RS + q]) =
                make_float4(racc[m][0] - yv[m][0], racc[m][1] - yv[m][1], racc[m][2] - yv[m][2], racc[m][3] - yv[m][3]);
    }
    __syncthreads();
    // rows pass 2: hr[p][q] = sum_v cT[v] r[p][q + v], p < RB MR, q < TW (over hx's buffer)
    if (t < TQ * B2) {
        const int sq = 4 * (t % TQ), sp = M2 * (t / TQ);
#pragma unroll
        for (int m = 0; m < M2; ++m) {
            if (sp + m >= RB * MR) break;
            float row[SEG * 4];
            bl_load_row<SEG>(&bufA[(sp + m) * RS + sq], row);
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int v = 0; v < K; ++v)
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] = __builtin_fmaf(a.scorr_c[v], row[k + v], acc[k]);
            *reinterpret_cast<float4*>(&bufB[(sp + m) * HS + sq]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
    }
    __syncthreads();
    // cols pass 2: g = -(sum_u rT[u] hr[p + u][q]) / sigma2 on the tile (+ the fused Langevin update)
    const int gq = 4 * (t % TQ), gp0 = BL_MG * (t / TQ);
    const int j = j0 + gq;
    if (j >= W || i0 + gp0 >= H) return;
    float acc[BL_MG][4];
#pragma unroll
    for (int m = 0; m < BL_MG; ++m) acc[m][0] = acc[m][1] = acc[m][2] = acc[m][3] = 0.f;
#pragma unroll
    for (int ir = 0; ir < BL_MG + 2 * L; ++ir) {
        const float4 v4 = *reinterpret_cast<const float4*>(&bufB[(gp0 + ir) * HS + gq]);
        const float hv[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
        for (int m = 0; m < BL_MG; ++m) {
            const int u = ir - m;
            if (u < 0 || u >= K) continue;
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[m][k] = __builtin_fmaf(a.scorr_r[u], hv[k], acc[m][k]);
        }
    }
#pragma unroll
    for (int m = 0; m < BL_MG; ++m) {
        const int i = i0 + gp0 + m;
        if (i >= H) break;
        float gv[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) gv[kk] = (-acc[m][kk]) * a.inv_sigma2;
        const size_t e0 = (size_t)c * HW + (size_t)i * W + j;
        const size_t o = (size_t)b * a.C * HW + e0;
        if (a.Y) {
            float z[4];
            if (vec) {
                normal_quad(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step, TAG_LANGEVIN, (uint32_t)(e0 >> 2), z);
                const float4 xv = ld4(a.X + o);
                *reinterpret_cast<float4*>(a.Y + o) =
                    make_float4((xv.x + a.c1 * gv[0]) + a.c2 * z[0], (xv.y + a.c1 * gv[1]) + a.c2 * z[1],
                                (xv.z + a.c1 * gv[2]) + a.c2 * z[2], (xv.w + a.c1 * gv[3]) + a.c2 * z[3]);
            } else {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    if (j + kk < W) {
                        const float zk = normal_elem(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step, TAG_LANGEVIN,
                                                     (uint64_t)(e0 + kk));
                        a.Y[o + kk] = (a.X[o + kk] + a.c1 * gv[kk]) + a.c2 * zk;
                    }
                }
            }
        } else if (vec) {
            *reinterpret_cast<float4*>(a.g + o) = make_float4(gv[0], gv[1], gv[2], gv[3]);
        } else {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
                if (j + kk < W) a.g[o + kk] = gv[kk];
        }
    }
}

static void launch_blur_sep(const BlurArgs& a, int l, dim3 grid, hipStream_t st) {
    switch (l) {
#define PSGLA_BLUR_CASE(LL) case LL: hipLaunchKernelGGL((blur_sep_kernel<LL>), grid, dim3(BL_THREADS), 0, st, a); break;
        PSGLA_BLUR_CASE(0) PSGLA_BLUR_CASE(1) PSGLA_BLUR_CASE(2) PSGLA_BLUR_CASE(3) PSGLA_BLUR_CASE(4)
        PSGLA_BLUR_CASE(5) PSGLA_BLUR_CASE(6) PSGLA_BLUR_CASE(7) PSGLA_BLUR_CASE(8)
#undef PSGLA_BLUR_CASE
        default: break;
    }
}

// h (K x K, row-major) == r c^T to fp32 rounding?  Pivot on the largest tap: c = its row, r = its column / pivot.
static bool blur_rank1(const float* h, int K, float* r, float* c) {
    int us = 0, vs = 0;
    float amax = 0.f;
    for (int u = 0; u < K; ++u)
        for (int v = 0; v < K; ++v)
            if (std::fabs(h[u * K + v]) > amax) { amax = std::fabs(h[u * K + v]); us = u; vs = v; }
    if (!(amax > 0.f) || !std::isfinite(amax)) return false;
    const double p = h[us * K + vs];
    for (int v = 0; v < K; ++v) c[v] = h[us * K + v];
    for (int u = 0; u < K; ++u) r[u] = (float)((double)h[u * K + vs] / p);
    for (int u = 0; u < K; ++u)
        for (int v = 0; v < K; ++v)
            if (std::fabs((double)h[u * K + v] - (double)r[u] * (double)c[v]) > 4.0 * FLT_EPSILON * amax) return false;
    return true;
}

template <bool EXACT>
static void launch_blur(const BlurArgs& a, int l, dim3 grid, hipStream_t st) {
    switch (l) {
#define PSGLA_BLUR_CASE(LL) case LL: hipLaunchKernelGGL((blur_grad_kernel<EXACT, LL>), grid, dim3(BL_THREADS), 0, st, a); break;
        PSGLA_BLUR_CASE(0) PSGLA_BLUR_CASE(1) PSGLA_BLUR_CASE(2) PSGLA_BLUR_CASE(3) PSGLA_BLUR_CASE(4)
        PSGLA_BLUR_CASE(5) PSGLA_BLUR_CASE(6) PSGLA_BLUR_CASE(7) PSGLA_BLUR_CASE(8)
#undef PSGLA_BLUR_CASE
        default: break;
    }
}

struct AccArgs {
    int n_inter, nm;
    const float* coef;
    float* samples;
    long long samples_cap;
    float* blocks;
    float* blocks2;
    long long blocks_cap;
    const long long* d_step;
    long long off;
};

__device__ __forceinline__ void acc_elem(const AccArgs& s, long long step, size_t idx, size_t BE, float X,
                                         float* mean, float* sq) {
    if (s.nm >= 0 && mean != nullptr) {
        const int per = s.nm + 1;
        const int im = (int)(step % per);
        const float ca = s.coef[2 * im], cb = s.coef[2 * im + 1];
        float m, q;
        if (im == 0) {
            m = cb * X;
            q = cb * (X * X);
        } else {
            m = ca * mean[idx] + cb * X;
            q = ca * sq[idx] + cb * (X * X);
        }
        if (im == s.nm) {
            const long long blk = step / per;
            if (blk < s.blocks_cap) {
                s.blocks[(size_t)blk * BE + idx] = m;
                s.blocks2[(size_t)blk * BE + idx] = q;
            }
        } else {
            mean[idx] = m;
            sq[idx] = q;
        }
    }
    if (s.n_inter > 0 && s.samples != nullptr && (step % s.n_inter) == 0) {
        const long long k = step / s.n_inter;
        if (k < s.samples_cap) s.samples[(size_t)k * BE + idx] = X;
    }
}

// The schedule decisions of one step, hoisted out of the element loops.
struct AccStep {
    bool acc, first, blockend, sample;
    long long blk, sidx;
    float ca, cb;
};
__device__ __forceinline__ AccStep acc_step(const AccArgs& s, long long step, const float* mean) {
    AccStep a;
    a.acc = s.nm >= 0 && mean != nullptr;
    const int per = s.nm + 1;
    const int im = a.acc ? (int)(step % per) : 0;
    a.first = im == 0;
    a.blk = a.acc ? step / per : 0;
    a.blockend = a.acc && im == s.nm;
    a.ca = a.acc ? s.coef[2 * im] : 0.f;
    a.cb = a.acc ? s.coef[2 * im + 1] : 0.f;
    a.sample = s.n_inter > 0 && s.samples != nullptr && (step % s.n_inter) == 0;
    a.sidx = a.sample ? step / s.n_inter : 0;
    a.sample = a.sample && a.sidx < s.samples_cap;
    return a;
}
// acc_elem's arithmetic on 4 aligned elements (idx % 4 == 0, 16-B accesses)
__device__ __forceinline__ void acc_quad(const AccArgs& s, const AccStep& st, size_t idx, size_t BE, const float4& X,
                                         float* mean, float* sq) {
    if (st.acc) {
        const float xs[4] = {X.x, X.y, X.z, X.w};
        float m[4], q[4];
        if (st.first) {
#pragma unroll
            for (int k = 0; k < 4; ++k) { m[k] = st.cb * xs[k]; q[k] = st.cb * (xs[k] * xs[k]); }
        } else {
            const float4 mo = ld4(mean + idx), qo = ld4(sq + idx);
            const float ms[4] = {mo.x, mo.y, mo.z, mo.w}, qs[4] = {qo.x, qo.y, qo.z, qo.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                m[k] = st.ca * ms[k] + st.cb * xs[k];
                q[k] = st.ca * qs[k] + st.cb * (xs[k] * xs[k]);
            }
        }
        if (st.blockend) {
            if (st.blk < s.blocks_cap) {
                st4(s.blocks + (size_t)st.blk * BE + idx, m[0], m[1], m[2], m[3]);
                st4(s.blocks2 + (size_t)st.blk * BE + idx, q[0], q[1], q[2], q[3]);
            }
        } else {
            st4(mean + idx, m[0], m[1], m[2], m[3]);
            st4(sq + idx, q[0], q[1], q[2], q[3]);
        }
    }
    if (st.sample) st4(s.samples + (size_t)st.sidx * BE + idx, X.x, X.y, X.z, X.w);
}

// X = (1 - alpha) Y + alpha D ; accumulate   (restoration_algorithms.py:238-271)
__global__ void relax_accumulate_kernel(const float* Y, const float* D, float* X, float alpha,
                                        int B, long long E, float* mean, float* sq, AccArgs s) {
    const long long step = read_step(s.d_step, s.off);
    const size_t BE = (size_t)B * E;
    if ((BE & 3) == 0) {
        const AccStep st = acc_step(s, step, mean);
        for (size_t i = 4 * (blockIdx.x * (size_t)blockDim.x + threadIdx.x); i < BE;
             i += 4 * (size_t)gridDim.x * blockDim.x) {
            const float4 y = ld4(Y + i), d = ld4(D + i);
            const float4 x = make_float4((1.0f - alpha) * y.x + alpha * d.x, (1.0f - alpha) * y.y + alpha * d.y,
                                         (1.0f - alpha) * y.z + alpha * d.z, (1.0f - alpha) * y.w + alpha * d.w);
            st4(X + i, x.x, x.y, x.z, x.w);
            acc_quad(s, st, i, BE, x, mean, sq);
        }
        return;
    }
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < BE;
         i += (size_t)gridDim.x * blockDim.x) {
        const float x = (1.0f - alpha) * Y[i] + alpha * D[i];
        X[i] = x;
        acc_elem(s, step, i, BE, x, mean, sq);
    }
}

// The DNN-denoiser PSGLA step's epilogue + the next step's prologue in one pass ("V-DnCNN"):
//   X = (1 - alpha) Y + alpha D ; samples / accumulators of step i  (restoration_algorithms.py:238-271)
//   Y' = (X + c1 g(X)) + c2 Z_{i+1},  g = ((-m)(X - y)) / sigma2    (:232-236, sampling_images.py:295)
// X itself is written only when X_out != nullptr (the next relaxation needs Y' and D', not X).
// Bit-identical to relax_accumulate + inpaint_grad + langevin_update (same operations, same order).
// grid: (quads of a plane, plane)
__global__ void relax_langevin_inpaint_kernel(const float* Y, const float* D, float* X_out, float alpha, int alpha1,
                                              const float* y, long long y_cs, const uint8_t* mask, long long m_cs,
                                              float* Y_next, int B, int C, int H, int W, float sigma2, float c1,
                                              float c2, unsigned long long seed, int chain0, float* mean, float* sq,
                                              AccArgs s) {
    const long long step = read_step(s.d_step, s.off);
    const size_t HW = (size_t)H * W;
    const size_t E = (size_t)C * HW;
    const size_t BE = (size_t)B * E;
    const int plane = blockIdx.y, b = plane / C, c = plane - b * C;
    const size_t p0 = (size_t)plane * HW;
    const float* yp = y + (size_t)b * y_cs + (size_t)c * HW;
    const uint8_t* mp = mask + (size_t)b * m_cs;
    const AccStep st = acc_step(s, step, mean);
    for (size_t i = 4 * (blockIdx.x * (size_t)blockDim.x + threadIdx.x); i < HW;
         i += 4 * (size_t)gridDim.x * blockDim.x) {
        const size_t idx = p0 + i;
        const float4 d = ld4(D + idx);
        float4 x = d;
        if (!alpha1) {
            const float4 yy = ld4(Y + idx);
            x = make_float4((1.0f - alpha) * yy.x + alpha * d.x, (1.0f - alpha) * yy.y + alpha * d.y,
                            (1.0f - alpha) * yy.z + alpha * d.z, (1.0f - alpha) * yy.w + alpha * d.w);
        }
        if (X_out) st4(X_out + idx, x.x, x.y, x.z, x.w);
        acc_quad(s, st, idx, BE, x, mean, sq);
        const float4 yo = ld4(yp + i);
        const uint32_t m = *reinterpret_cast<const uint32_t*>(mp + i);
        const float m0 = (float)(m & 0xFFu), m1 = (float)((m >> 8) & 0xFFu), m2 = (float)((m >> 16) & 0xFFu),
                    m3 = (float)(m >> 24);
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)(step + 1), TAG_LANGEVIN,
                    (uint32_t)(((size_t)c * HW + i) >> 2), z);
        const float g0 = (-m0 * (x.x - yo.x)) / sigma2, g1 = (-m1 * (x.y - yo.y)) / sigma2,
                    g2 = (-m2 * (x.z - yo.z)) / sigma2, g3 = (-m3 * (x.w - yo.w)) / sigma2;
        st4(Y_next + idx, (x.x + c1 * g0) + c2 * z[0], (x.y + c1 * g1) + c2 * z[1], (x.z + c1 * g2) + c2 * z[2],
            (x.w + c1 * g3) + c2 * z[3]);
    }
}

// The same pass for H*W % 4 != 0 (set1c / CBSD68 are 481 x 321): chain-linear quads, so the noise
// quad of an element is the one psgla_langevin_update gives it (e >> 2 of the chain's C*H*W image);
// scalar loads, one element at a time.  grid: (quads of a chain, chain)
__global__ void relax_langevin_inpaint_any_kernel(const float* Y, const float* D, float* X_out, float alpha,
                                                  int alpha1, const float* y, long long y_cs, const uint8_t* mask,
                                                  long long m_cs, float* Y_next, int B, int C, int H, int W,
                                                  float sigma2, float c1, float c2, unsigned long long seed,
                                                  int chain0, float* mean, float* sq, AccArgs s) {
    const long long step = read_step(s.d_step, s.off);
    const long long HW = (long long)H * W;
    const long long E = (long long)C * HW;
    const size_t BE = (size_t)B * E;
    const int b = blockIdx.y;
    const float* yp = y + (size_t)b * y_cs;
    const uint8_t* mp = mask + (size_t)b * m_cs;
    const long long Q = (E + 3) >> 2;
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < Q; q += (long long)gridDim.x * blockDim.x) {
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)(step + 1), TAG_LANGEVIN, (uint32_t)q, z);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const long long e = 4 * q + j;
            if (e >= E) break;
            const size_t idx = (size_t)b * E + e;
            const float x = alpha1 ? D[idx] : (1.0f - alpha) * Y[idx] + alpha * D[idx];
            if (X_out) X_out[idx] = x;
            acc_elem(s, step, idx, BE, x, mean, sq);
            const float m = (float)mp[e % HW];
            const float g = (-m * (x - yp[e])) / sigma2;
            Y_next[idx] = (x + c1 * g) + c2 * z[j];
        }
    }
}

// PnP-ULA (restoration_algorithms.py:104-115)
__global__ void pnpula_update_kernel(const float* X, const float* gp, const float* gd, float* Xo,
                                     float delta, float lambd, float brw, float cmin, float cmax, int B,
                                     long long E, float* mean, float* sq, unsigned long long seed,
                                     int chain0, AccArgs s) {
    // grid: (quads of a chain, chain)
    const long long step = read_step(s.d_step, s.off);
    const long long Q = (E + 3) >> 2;
    const size_t BE = (size_t)B * E;
    const int b = blockIdx.y;
    const bool vec = (E & 3) == 0;
    const AccStep st = acc_step(s, step, mean);
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < Q;
         q += (long long)gridDim.x * blockDim.x) {
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)step, TAG_LANGEVIN, (uint32_t)q, z);
        const size_t i0 = (size_t)b * E + (size_t)(q << 2);
        auto upd = [&](float x, float gpv, float gdv, float zz) {
            const float out = (x > cmin) ? x : cmin;
            const float proj = (out < cmax) ? out : cmax;
            const float gpi = (gpv - (x - proj) / lambd) + gdv;
            return (x + delta * gpi) + brw * zz;
        };
        if (vec) {
            const float4 x = ld4(X + i0), p4 = ld4(gp + i0), d4 = ld4(gd + i0);
            const float4 xn = make_float4(upd(x.x, p4.x, d4.x, z[0]), upd(x.y, p4.y, d4.y, z[1]),
                                          upd(x.z, p4.z, d4.z, z[2]), upd(x.w, p4.w, d4.w, z[3]));
            st4(Xo + i0, xn.x, xn.y, xn.z, xn.w);
            acc_quad(s, st, i0, BE, xn, mean, sq);
        } else {
            for (int j = 0; j < 4; ++j) {
                if ((q << 2) + j >= E) break;
                const size_t i = i0 + j;
                const float xn = upd(X[i], gp[i], gd[i], z[j]);
                Xo[i] = xn;
                acc_elem(s, step, i, BE, xn, mean, sq);
            }
        }
    }
}

// PnP-ULA step with the DNN prior fused ("V-ULA", restoration_algorithms.py:104-115 with the prior of
// sampling_images.py:156-157): gp = (alpha (D - X)) / s2 from the denoiser output D = D(X, s1), the
// inpainting data term gd = ((-m)(X - y)) / sigma2 computed in place (gd == nullptr) or a given gd
// (deblurring: the stencil kernel's output), the projection, the update, the noise and the
// accumulators in one pass -- read X, D, y, mean, sq (+ the shared mask), write X', mean, sq: 32 B/elem.
// The same fp32 operations, in the same order, as DenoiserPrior's torch ops + psgla_inpaint_grad +
// pnpula_update.  grid: (quads of a chain, chain); quads are chain-linear (the noise quads).
__global__ void pnpula_prior_update_kernel(const float* X, const float* D, float alpha, float s2, const float* gd,
                                           const float* y, long long y_cs, const uint8_t* mask, long long m_cs,
                                           float sigma2, float* Xo, float delta, float lambd, float brw, float cmin,
                                           float cmax, int B, long long HW, long long E, float* mean, float* sq,
                                           unsigned long long seed, int chain0, AccArgs s) {
    const long long step = read_step(s.d_step, s.off);
    const long long Q = (E + 3) >> 2;
    const size_t BE = (size_t)B * E;
    const int b = blockIdx.y;
    const bool vec = (E & 3) == 0 && (HW & 3) == 0;
    const AccStep st = acc_step(s, step, mean);
    const float* yp = y ? y + (size_t)b * y_cs : nullptr;
    const uint8_t* mp = mask ? mask + (size_t)b * m_cs : nullptr;
    auto upd = [&](float x, float d, float gdv, float zz) {
        const float gpv = (alpha * (d - x)) / s2;
        const float out = (x > cmin) ? x : cmin;
        const float proj = (out < cmax) ? out : cmax;
        const float gpi = (gpv - (x - proj) / lambd) + gdv;
        return (x + delta * gpi) + brw * zz;
    };
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < Q;
         q += (long long)gridDim.x * blockDim.x) {
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)step, TAG_LANGEVIN, (uint32_t)q, z);
        const size_t i0 = (size_t)b * E + (size_t)(q << 2);
        if (vec) {
            const float4 x = ld4(X + i0), d = ld4(D + i0);
            float g[4];
            if (gd) {
                const float4 g4 = ld4(gd + i0);
                g[0] = g4.x; g[1] = g4.y; g[2] = g4.z; g[3] = g4.w;
            } else {
                const long long e = q << 2;
                const float4 yy = ld4(yp + e);
                const uint32_t m = *reinterpret_cast<const uint32_t*>(mp + (e % HW));
                g[0] = (-(float)(m & 0xFFu) * (x.x - yy.x)) / sigma2;
                g[1] = (-(float)((m >> 8) & 0xFFu) * (x.y - yy.y)) / sigma2;
                g[2] = (-(float)((m >> 16) & 0xFFu) * (x.z - yy.z)) / sigma2;
                g[3] = (-(float)(m >> 24) * (x.w - yy.w)) / sigma2;
            }
            const float4 xn = make_float4(upd(x.x, d.x, g[0], z[0]), upd(x.y, d.y, g[1], z[1]),
                                          upd(x.z, d.z, g[2], z[2]), upd(x.w, d.w, g[3], z[3]));
            st4(Xo + i0, xn.x, xn.y, xn.z, xn.w);
            acc_quad(s, st, i0, BE, xn, mean, sq);
        } else {
            for (int j = 0; j < 4; ++j) {
                const long long e = (q << 2) + j;
                if (e >= E) break;
                const size_t i = i0 + j;
                const float x = X[i];
                const float gdv = gd ? gd[i] : (-(float)mp[e % HW] * (x - yp[e])) / sigma2;
                const float xn = upd(x, D[i], gdv, z[j]);
                Xo[i] = xn;
                acc_elem(s, step, i, BE, xn, mean, sq);
            }
        }
    }
}

// DnCNN layer epilogue (denoisers.py DnCNN, deepinv's conv -> bias -> ReLU): y = relu(y + bias[c]) in
// place, one pass instead of PyTorch's bias add and ReLU passes over a 1 GB activation tensor at 64
// chains.  NHWC (hw == 0: c = e % C, C % 4 == 0) or NCHW (c = (e / hw) % C, hw % 4 == 0).  ReLU as
// (v < 0) ? 0 : v -- PyTorch's clamp_min(0): NaN and -0 pass through unchanged.
__global__ void bias_act_kernel(float* y, const float* bias, long long n4, int C, long long hw, int relu) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const long long e = 4 * i;
        float4 v = ld4(y + e);
        float4 bb;
        if (hw == 0) {
            bb = ld4(bias + (int)(e % C));
        } else {
            const float b1 = bias[(int)((e / hw) % C)];
            bb = make_float4(b1, b1, b1, b1);
        }
        v.x = v.x + bb.x; v.y = v.y + bb.y; v.z = v.z + bb.z; v.w = v.w + bb.w;
        if (relu) {
            v.x = v.x < 0.f ? 0.f : v.x; v.y = v.y < 0.f ? 0.f : v.y;
            v.z = v.z < 0.f ? 0.f : v.z; v.w = v.w < 0.f ? 0.f : v.w;
        }
        st4(y + e, v.x, v.y, v.z, v.w);
    }
}

// g = ((-m) (X - y)) / sigma2   (sampling_images.py:295)
__global__ void inpaint_grad_kernel(const float* X, const float* y, long long y_cs, const uint8_t* mask,
                                    long long m_cs, float* g, int B, int C, int H, int W, float sigma2) {
    // grid: (quads of a plane, plane)
    const size_t HW = (size_t)H * W;
    const int plane = blockIdx.y, b = plane / C, c = plane - b * C;
    const float* xp = X + (size_t)plane * HW;
    const float* yp = y + (size_t)b * y_cs + (size_t)c * HW;
    const uint8_t* mp = mask + (size_t)b * m_cs;
    float* gq = g + (size_t)plane * HW;
    if ((HW & 3) == 0) {
        for (size_t i = 4 * (blockIdx.x * (size_t)blockDim.x + threadIdx.x); i < HW;
             i += 4 * (size_t)gridDim.x * blockDim.x) {
            const float4 x = ld4(xp + i), yy = ld4(yp + i);
            const uint32_t m = *reinterpret_cast<const uint32_t*>(mp + i);
            const float m0 = (float)(m & 0xFFu), m1 = (float)((m >> 8) & 0xFFu), m2 = (float)((m >> 16) & 0xFFu),
                        m3 = (float)(m >> 24);
            st4(gq + i, (-m0 * (x.x - yy.x)) / sigma2, (-m1 * (x.y - yy.y)) / sigma2,
                (-m2 * (x.z - yy.z)) / sigma2, (-m3 * (x.w - yy.w)) / sigma2);
        }
        return;
    }
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < HW; i += (size_t)gridDim.x * blockDim.x) {
        const float m = (float)mp[i];
        gq[i] = (-m * (xp[i] - yp[i])) / sigma2;
    }
}

__global__ void advance_step_kernel(long long* d) { *d = *d + 1; }

// Diagnostic: the Box-Muller radius / angle for 24-bit indices [k0, k0+n) (exhaustive noise test).
__global__ void bm_tables_kernel(float* r, float* cs, float* sn, uint32_t k0, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t k = k0 + i;
        r[i] = bm_radius(k);
        float c, s;
        bm_angle(k, c, s);
        cs[i] = c;
        sn[i] = s;
    }
}

}  // namespace psgla

// =======================================================================================
// C ABI
// =======================================================================================
using namespace psgla;

static thread_local char g_err[512] = "";

static int fail(int code, const char* msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
    return code ? code : (int)hipErrorInvalidValue;
}

static int launch_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return 0;
}

// x-extent of a (work items of one chain / plane, chains) grid: ~4 waves of workgroups over the CUs
static int grid_chain(long long per_chain, int chains) {
    long long g = (per_chain + 255) / 256;
    const long long cap = (4LL * 256 + chains - 1) / chains;   // total ~ 4 x 256 CUs x ... workgroups
    if (g > cap * 4) g = cap * 4;
    if (g < 1) g = 1;
    return (int)g;
}

static int grid_for(long long n, int threads) {
    long long g = (n + threads - 1) / threads;
    if (g > 256 * 16) g = 256 * 16;
    if (g < 1) g = 1;
    return (int)g;
}

static void tv_tiling(TvArgs& a) {
    const int h = a.halo;
    if (a.H <= TV_ROWS) {
        a.band_h = a.H; a.nbands = 1;
    } else {
        const int bh = TV_ROWS - 2 * h;
        a.nbands = (a.H + bh - 1) / bh;
        a.band_h = (a.H + a.nbands - 1) / a.nbands;
    }
    if (a.W <= TV_COLS) {
        a.seg_w = a.W; a.nsegs = 1;
    } else {
        const int sw = (TV_COLS - 2 * h - 3) & ~3;
        a.nsegs = (a.W + sw - 1) / sw;
        a.seg_w = (((a.W + a.nsegs - 1) / a.nsegs) + 3) & ~3;
    }
    a.tiles = a.nbands * a.nsegs;
}

static int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) return 256;
    return cus;
}

// Row-split workgroup count for the streaming kernel (0 = one workgroup per plane).
// req: 0 auto, -1 per plane, > 0 forced.  A range of R rows touches at most ceil(R/H) + 1
// planes, so R <= 3H keeps it within SP_MAXSEG = 4 segments: G >= ceil(P/3).
// P: (virtual) planes = B * C * column segments, each of H rows
static int choose_split(long long P, int H, int h, int req, int* out) {
    const long long T = P * H;
    const long long gmin = (P + SP_MAXSEG - 2) / (SP_MAXSEG - 1);
    *out = 0;
    if (req < 0) return 0;
    if (req > 0) {
        if (req < gmin || req > T) return fail(0, "psgla_tv_step: stream_wgs outside [ceil(P/3), P*H]");
        *out = req;
        return 0;
    }
    const long long cus = device_cus();
    if (P > (SP_MAXSEG - 1) * cus) return 0;          // enough planes: one workgroup each
    long long g = (T + 4LL * h - 1) / (4LL * h);      // >= 4 n_tv core rows per range
    if (g > cus) g = cus;
    if (g < gmin) g = gmin;
    if (g <= P && T % g == 0 && (T / g) % H == 0) return 0;   // ranges = whole planes anyway
    *out = (int)g;
    return 0;
}

// Small-batch tile kernel geometry: NW waves of R rows (tile = NW R rows incl. n_tv halo rows at cuts
// inside a plane), equal bands per plane, nsegs column segments (stream_segments); a band's core rows
// stay within the LDS staging of mean / sq (tile_mst_rows).  Returns the number of workgroups (tiles
// rounded up to 8 -- the XCD-aware order), 0 if the shape does not fit (halo too large, no segmentation).
static int tile_geometry(int P, int H, int nsegs, int h, int NW, int R, int* band_h, int* nbands) {
    if (nsegs < 1 || R < 2) return 0;
    const int rows = NW * R, mst = tile_mst_rows(NW, R);
    int nb, bh;
    if (H <= mst) {
        nb = 1; bh = H;
    } else {
        const int core = min(rows - 2 * h, mst);
        if (core < 1) return 0;
        nb = (H + core - 1) / core;
        bh = (H + nb - 1) / nb;
    }
    *band_h = bh;
    *nbands = nb;
    return ((P * nb * nsegs + 7) / 8) * 8;
}

// Column segments of the streaming kernel: equal core widths (multiples of 4) cut from the image
// width W; segment s's wave covers columns [f0, f0 + 256) with f0 = (cc0 - h) & ~3 (cc0 = s * seg_w),
// which must reach cc1 + h for interior cuts (the TV dependency cone) and the row pitch L at the
// image's right end (no halo needed at the image edges).  Fewest segments; 0 if none fits.
static int stream_segments(int W, int L, int h, int* seg_w) {
    for (int n = 1; n <= 64; ++n) {
        const int sw = (((W + n - 1) / n) + 3) & ~3;
        if ((long long)sw * (n - 1) >= W) continue;         // last segment would be empty
        bool ok = true;
        for (int sgi = 0; sgi < n && ok; ++sgi) {
            const int cc0 = sgi * sw, cc1 = min(W, cc0 + sw);
            const int f0 = max(0, cc0 - h) & ~3;
            const int need = (cc1 >= W) ? L : min(L, cc1 + h);
            ok = need - f0 <= TV_COLS;
        }
        if (ok) {
            if (seg_w) *seg_w = sw;
            return n;
        }
    }
    return 0;
}

template <bool EXACT, int FRONT, bool ALPHA1>
static int launch_tv(const TvArgs& a, hipStream_t st, int mask = 3) {
    const int P = a.B * a.C;
    if (mask == 0) mask = 3;
    if (mask & 1) {
        if (FRONT == FRONT_INPAINT && a.tile_r > 0) {
            TvArgs s = a;
            s.fin_inline = (mask & 2) ? 1 : 0;
            const int grid = ((P * s.nbands * s.st_nsegs + 7) / 8) * 8;   // tile_kernel: 8 runs of tiles
            // (the two-phase arrival counter keeps a count of workgroups in 15 bits)
            if (grid > 32767) return fail(0, "psgla_tv_step: more than 32767 tiles in one launch");
            // several copies of the rel-err sums only where many tiles share a chain (castle at B = 1: 246 tiles,
            // 34.8 -> 33.0 us); with 15-66 tiles per chain the last workgroup's reads of 8 copies cost more
            // (+4-5 %) than the queueing they save (profiles/r03s_tile_norm_copies_ab.txt)
            if (s.norm_copies < 1 || s.C * s.nbands * s.st_nsegs < 128) s.norm_copies = 1;
            const bool gen = !(s.ldw == s.W && s.st_nsegs == 1);
#define PSGLA_TILE(NWV, RV)                                                                                        \
    if (s.tile_nw == NWV && s.tile_r == RV) {                                                                      \
        if (!gen) hipLaunchKernelGGL((tv_tile_kernel<EXACT, ALPHA1, RV, false, NWV>), dim3(grid), dim3(NWV * WAVE), 0, st, s); \
        else hipLaunchKernelGGL((tv_tile_kernel<EXACT, ALPHA1, RV, true, NWV>), dim3(grid), dim3(NWV * WAVE), 0, st, s);       \
        return launch_check("tv_tile_kernel");                                                                     \
    }
            PSGLA_TILE(16, 2)
            PSGLA_TILE(16, 3)
            PSGLA_TILE(8, 4)
            PSGLA_TILE(8, 6)
            PSGLA_TILE(8, 9)
#undef PSGLA_TILE
            return fail(0, "psgla_tv_step: internal error: no tile kernel of this shape");
        }
        if (FRONT == FRONT_INPAINT && a.stream) {
            TvArgs s = a;
            s.fin_inline = (mask & 2) ? 1 : 0;
            const int grid = s.split_wgs > 0 ? s.split_wgs : P * s.st_nsegs;   // virtual planes
            const bool gen = !(s.ldw == s.W && s.st_nsegs == 1);
            if (!gen)
                hipLaunchKernelGGL((tv_stream_kernel<EXACT, ALPHA1, false>), dim3(grid), dim3(TV_THREADS), 0, st, s);
            else
                hipLaunchKernelGGL((tv_stream_kernel<EXACT, ALPHA1, true>), dim3(grid), dim3(TV_THREADS), 0, st, s);
            int rc = launch_check("tv_stream_kernel");
            if (rc) return rc;
            return 0;                    // finalised in-kernel (or main pass only)
        } else {
            const int grid_main = ((P + 7) / 8) * 8 * a.tiles;
            hipLaunchKernelGGL((tv_main_kernel<EXACT, FRONT, ALPHA1>), dim3(grid_main), dim3(TV_THREADS), 0, st, a);
        }
        int rc = launch_check("tv_kernel(main)");
        if (rc) return rc;
    }
    if (!(mask & 2)) return 0;
    // Few workgroups: every one re-derives the per-chain stop flags (cheap) and they meet on one
    // arrival counter -- 8 contending atomics instead of one per CU (measured 13.5 us -> see
    // DESIGN.md).  The rare early-stop recompute is spread over these workgroups.
    const int grid_fin = (P * a.tiles < 8) ? P * a.tiles : 8;
    hipLaunchKernelGGL((tv_finalise_kernel<EXACT, FRONT, ALPHA1>), dim3(grid_fin), dim3(TV_THREADS), 0, st, a);
    return launch_check("tv_kernel(finalise)");
}

static int check_tv_common(int B, int C, int H, int W, int n_tv) {
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return fail(0, "psgla: empty tensor dimensions");
    if (B > MAXG) return fail(0, "psgla: more than 1024 chains in one launch; split the batch");
    if (n_tv < 0 || n_tv > MAXIT)
        return fail(0, "psgla: n_it_max outside [0, PSGLA_TV_MAX_FUSED_IT] for the fused TV kernel");
    if (H > TV_ROWS && TV_ROWS - 2 * n_tv < 1) return fail(0, "psgla: TV halo too large");
    return 0;
}

// Which fused-step kernel psgla_tv_step launches for a descriptor, and its geometry in `a` (B, C, H, W,
// ldw and n_tv of `a` set): 0 band kernel (+ finaliser), 1 row stream, 3 small-batch tile kernel; -1 with
// g_sel_err on a shape the requested variant does not support.
static thread_local const char* g_sel_err = "";
static int select_step_kernel(const PsglaTvStep* d, TvArgs& a) {
    a.halo = d->n_tv;
    tv_tiling(a);
    const bool streamable = (a.ldw % 4 == 0) && d->n_tv >= 1 && d->n_tv <= SP_MAXST && d->H >= 2 &&
                            stream_segments(a.W, a.ldw, d->n_tv, nullptr) > 0;
    a.stream = streamable && d->kernel_variant != 1;
    if (d->kernel_variant == 2 && !streamable)
        { g_sel_err = "psgla_tv_step: shape not supported by the streaming kernel"; return -1; }
    if (d->kernel_variant < 0 || d->kernel_variant > 4 || d->kernel_variant == 3)
        { g_sel_err = "psgla_tv_step: kernel_variant must be 0 (auto), 1 (band), 2 (stream) or 4 (tile)"; return -1; }
    // small-batch tile kernel: forced (variant 4) or, in auto mode, when all tiles fit in one round
    // on the CUs (a row stream would be mostly pipeline fill: strong scaling's 64/N chains per GPU)
    a.tile_r = 0;
    a.tile_nw = 16;
    int tile_segs = 0, tile_sw = 0;
    if (d->kernel_variant == 4 || d->kernel_variant == 0) {
        const int P = d->B * d->C;
        int bh = 0, nb = 0;
        // column segments as the stream kernel's (one when ldw == W <= 256)
        tile_segs = (a.ldw % 4 == 0 && d->n_tv >= 1) ? stream_segments(a.W, a.ldw, d->n_tv, &tile_sw) : 0;
        int bh2 = 0, nb2 = 0, bh9 = 0, nb9 = 0;
        const int wg = tile_geometry(P, d->H, tile_segs, d->n_tv, 16, 3, &bh, &nb);
        const int wg2 = tile_geometry(P, d->H, tile_segs, d->n_tv, 16, 2, &bh2, &nb2);
        const int wg9 = tile_geometry(P, d->H, tile_segs, d->n_tv, 8, 9, &bh9, &nb9);
        if (d->kernel_variant == 4 && wg == 0) { g_sel_err = "psgla_tv_step: shape not supported by the tile kernel"; return -1; }
        // auto: the tiles fit in one round on the CUs -- or in two when the rows need column segments (W > 256),
        // where the row stream's 256-column windows run a third of their lanes idle (measured: castle-size
        // images at B = 3-4 and 321 x 481 at B = 4-6 run faster as two rounds of tiles; 256 x 256 does not,
        // profiles/r03l_tile_threshold.txt)
        const long long ntiles = (long long)P * nb * tile_segs, cus = device_cus();
        const long long ntiles9 = (long long)P * nb9 * tile_segs;
        if (wg > 0 && (d->kernel_variant == 4 || ntiles <= cus || (wg9 > 0 && ntiles9 <= cus) ||
                       (tile_segs > 1 && ntiles <= 2 * cus))) {
            a.tile_r = 3;
            a.tile_nw = 16;
            a.band_h = bh;
            a.nbands = nb;
            // 72-row tiles (8 waves x 9 rows) when 48-row tiles would need a second round but these fit in one
            if (ntiles > cus && wg9 > 0 && ntiles9 <= cus) {
                a.tile_r = 9;
                a.tile_nw = 8;
                a.band_h = bh9;
                a.nbands = nb9;
            }
            // 32-row tiles (2 rows per wave) when they still fit in one round: one or a few images leave most
            // CUs idle at 48 rows (castle B = 1: 114 tiles of 48 rows vs 246 of 32 rows, 41.1 -> 35.0 us,
            // profiles/r03q_tile_r2_ab.txt); more tiles but shorter waves
            if (wg2 > 0 && (long long)P * nb2 * tile_segs <= cus) {
                a.tile_r = 2;
                a.tile_nw = 16;
                a.band_h = bh2;
                a.nbands = nb2;
            }
            a.nsegs = 1;
            a.tiles = a.nbands * tile_segs;
            a.stream = 0;
        }
    }
    if (!a.stream && a.tile_r == 0 && a.ldw != a.W) { g_sel_err = "psgla_tv_step: a row pitch ldw != W needs the streaming or the tile kernel"; return -1; }
    a.split_wgs = 0;
    a.st_nsegs = 1;
    if (a.tile_r > 0) {
        a.st_nsegs = tile_segs;
        a.st_seg_w = tile_sw;
        a.st_halo = d->n_tv;
    }
    if (a.stream) {
        a.st_halo = d->n_tv;
        a.st_nsegs = stream_segments(a.W, a.ldw, d->n_tv, &a.st_seg_w);
        if (choose_split((long long)d->B * d->C * a.st_nsegs, d->H, d->n_tv, d->stream_wgs, &a.split_wgs)) {
            g_sel_err = g_err;
            return -1;
        }
    }
    if (a.tile_r > 0) return 3;
    if (a.stream) return 1;
    return 0;
}

extern "C" {

int psgla_abi_version(void) { return PSGLA_HIP_ABI_VERSION; }
const char* psgla_last_error(void) { return g_err; }

int psgla_tv_step(const PsglaTvStep* d, const PsglaSchedule* s, void* stream) {
    if (!d || !s) return fail(0, "psgla_tv_step: null descriptor");
    int rc = check_tv_common(d->B, d->C, d->H, d->W, d->n_tv);
    if (rc) return rc;
    const bool alpha1 = d->x2[0] == nullptr;
    if (!d->x[0] || !d->x[1] || !d->u2[0] || !d->u2[1] || !d->y || !d->mask || !d->norms || !d->arrive ||
        !d->fresh)
        return fail(0, "psgla_tv_step: missing buffer");
    if (!alpha1 && !d->x2[1]) return fail(0, "psgla_tv_step: x2[1] missing");
    if (s->n_inter_mmse >= 0 && (!d->mean[0] || !d->mean[1] || !d->sq[0] || !d->sq[1] || !s->acc_coef))
        return fail(0, "psgla_tv_step: accumulators missing");
    TvArgs a;
    memset(&a, 0, sizeof(a));
    a.B = d->B; a.C = d->C; a.H = d->H; a.W = d->W;
    a.ldw = d->ldw > 0 ? d->ldw : d->W;
    if (a.ldw < a.W) return fail(0, "psgla_tv_step: ldw < W");
    for (int i = 0; i < 2; ++i) {
        a.x[i] = d->x[i]; a.u2[i] = d->u2[i]; a.x2[i] = d->x2[i]; a.mean[i] = d->mean[i]; a.sq[i] = d->sq[i];
    }
    a.yobs = d->y; a.y_cs = d->y_chain_stride; a.mask = d->mask; a.m_cs = d->mask_chain_stride;
    a.c1 = d->c1; a.c2 = d->c2; a.sigma2 = d->sigma2; a.alpha = d->alpha;
    a.tau = d->tau; a.opt = d->one_plus_tau; a.inv_opt = (float)(1.0 / (double)d->one_plus_tau);
    a.sig_tv = d->sigma_tv; a.rho = d->rho; a.ths = d->ths; a.tol = d->tol;
    a.inv_sigma2 = (float)(1.0 / (double)a.sigma2);
    a.n_tv = d->n_tv; a.seed = d->seed; a.chain0 = d->chain0; a.pingpong = 1;
    a.d_step = (long long*)s->d_step; a.step_offset = s->step_offset;
    a.fresh_dev = d->fresh; a.per_chain_norm = 1; a.norms = d->norms; a.arrive = d->arrive;
    a.norm_copies = d->norms_copies > 1 ? d->norms_copies : 1;
    a.it0 = 0; a.last_chunk = 1; a.stopped = nullptr;
    a.advance_step = d->advance_step;
    a.n_inter = s->n_inter; a.nm = s->n_inter_mmse; a.coef = s->acc_coef;
    a.samples = s->samples; a.samples_cap = s->samples_cap;
    a.blocks = s->blocks; a.blocks2 = s->blocks2; a.blocks_cap = s->blocks_cap;
    if (select_step_kernel(d, a) < 0) return g_sel_err == g_err ? (int)hipErrorInvalidValue : fail(0, g_sel_err);
    hipStream_t st = (hipStream_t)stream;
    const int m = d->launch_mask;
    if (d->exact)
        return alpha1 ? launch_tv<true, FRONT_INPAINT, true>(a, st, m) : launch_tv<true, FRONT_INPAINT, false>(a, st, m);
    return alpha1 ? launch_tv<false, FRONT_INPAINT, true>(a, st, m) : launch_tv<false, FRONT_INPAINT, false>(a, st, m);
}

int psgla_tv_step_kernel(const PsglaTvStep* d) {
    if (!d) return fail(0, "psgla_tv_step_kernel: null descriptor");
    const int rc = check_tv_common(d->B, d->C, d->H, d->W, d->n_tv);
    if (rc) return -1;
    TvArgs a;
    memset(&a, 0, sizeof(a));
    a.B = d->B; a.C = d->C; a.H = d->H; a.W = d->W;
    a.ldw = d->ldw > 0 ? d->ldw : d->W;
    const int k = select_step_kernel(d, a);
    if (k < 0 && g_sel_err != g_err) fail(0, g_sel_err);
    return k;
}

int psgla_tv_prox(const PsglaTvProx* d, void* stream) {
    if (!d) return fail(0, "psgla_tv_prox: null descriptor");
    int rc = check_tv_common(d->B, d->C, d->H, d->W, d->n_tv);
    if (rc) return rc;
    if (!d->y || !d->x2_out || !d->u2_out || !d->norms || !d->arrive) return fail(0, "psgla_tv_prox: missing buffer");
    if (!d->fresh && (!d->x2_in || !d->u2_in)) return fail(0, "psgla_tv_prox: warm start needs x2_in/u2_in");
    TvArgs a;
    memset(&a, 0, sizeof(a));
    a.B = d->B; a.C = d->C; a.H = d->H; a.W = d->W;
    a.yin = d->y;
    a.x2[0] = const_cast<float*>(d->x2_in); a.x2[1] = d->x2_out;
    a.u2[0] = const_cast<float*>(d->u2_in); a.u2[1] = d->u2_out;
    a.tau = d->tau; a.opt = d->one_plus_tau; a.inv_opt = (float)(1.0 / (double)d->one_plus_tau);
    a.sig_tv = d->sigma_tv; a.rho = d->rho; a.ths = d->ths; a.tol = d->tol;
    a.n_tv = d->n_tv; a.pingpong = 0;
    a.fresh_host = d->fresh; a.per_chain_norm = d->per_chain ? 1 : 0; a.norms = d->norms; a.arrive = d->arrive;
    if (d->it0 < 0) return fail(0, "psgla_tv_prox: it0 < 0");
    a.it0 = d->it0; a.last_chunk = d->last_chunk ? 1 : 0; a.stopped = d->stopped;
    a.nm = -1;
    a.halo = d->n_tv;
    tv_tiling(a);
    hipStream_t st = (hipStream_t)stream;
    return d->exact ? launch_tv<true, FRONT_GIVEN, true>(a, st) : launch_tv<false, FRONT_GIVEN, true>(a, st);
}

int psgla_normal_fill(float* out, int32_t B, int64_t E, uint64_t seed, int32_t chain0, const int64_t* d_step,
                      int64_t step_offset, uint32_t tag, void* stream) {
    if (!out || B <= 0 || E <= 0) return fail(0, "psgla_normal_fill: bad arguments");
    const long long total = (long long)B * ((E + 3) / 4);
    hipLaunchKernelGGL(normal_fill_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, out, B,
                       (long long)E, (unsigned long long)seed, chain0, (const long long*)d_step,
                       (long long)step_offset, tag);
    return launch_check("normal_fill");
}

int psgla_langevin_update(const float* X, const float* g, float* Y, int32_t B, int64_t E, float c1, float c2,
                          uint64_t seed, int32_t chain0, const int64_t* d_step, int64_t step_offset,
                          void* stream) {
    if (!X || !g || !Y || B <= 0 || E <= 0) return fail(0, "psgla_langevin_update: bad arguments");
    const long long total = (long long)B * ((E + 3) / 4);
    if (B > 65535) return fail(0, "psgla_langevin_update: more than 65535 chains in one launch");
    hipLaunchKernelGGL(langevin_update_kernel, dim3(grid_chain(E / 4 + 1, B), B), dim3(256), 0, (hipStream_t)stream, X,
                       g, Y, B, (long long)E, c1, c2, (unsigned long long)seed, chain0,
                       (const long long*)d_step, (long long)step_offset);
    return launch_check("langevin_update");
}

// diagnostic switch (tests, A/B): 1 = fast mode always takes the 2-D kernel
static int g_blur_no_sep = 0;
extern "C" int psgla_blur_set_separable(int32_t enable) {
    g_blur_no_sep = enable ? 0 : 1;
    return 0;
}

int psgla_blur_grad(const float* X, const float* y, int64_t y_chain_stride, const float* hconv, const float* hcorr,
                    int32_t l, float* g, float* Y, int32_t B, int32_t C, int32_t H, int32_t W, float sigma2,
                    float c1, float c2, uint64_t seed, int32_t chain0, const int64_t* d_step, int64_t step_offset,
                    int32_t exact, void* stream) {
    if (!X || !y || !hconv || !hcorr || (!g && !Y) || B <= 0 || C <= 0 || H <= 0 || W <= 0)
        return fail(0, "psgla_blur_grad: bad arguments");
    if (l < 0 || l > BL_MAXL) return fail(0, "psgla_blur_grad: blur half-width l outside [0, 8]");
    if ((long long)B * C > 65535) return fail(0, "psgla_blur_grad: more than 65535 planes in one launch");
    BlurArgs a;
    memset(&a, 0, sizeof(a));
    const int K = 2 * l + 1;
    // the taps (HOST memory, like the scalars) travel as kernel arguments: SGPR operands
    memcpy(a.hconv, hconv, sizeof(float) * K * K);
    memcpy(a.hcorr, hcorr, sizeof(float) * K * K);
    a.X = X; a.y = y; a.y_cs = y_chain_stride; a.g = g; a.Y = Y;
    a.B = B; a.C = C; a.H = H; a.W = W; a.sigma2 = sigma2; a.inv_sigma2 = (float)(1.0 / (double)sigma2);
    a.c1 = c1; a.c2 = c2; a.seed = seed; a.chain0 = chain0; a.d_step = (const long long*)d_step;
    a.off = step_offset;
    a.tiles_x = (W + BL_TW - 1) / BL_TW;
    a.tiles_y = (H + BL_TH - 1) / BL_TH;
    const long long ntiles = (long long)a.tiles_x * a.tiles_y * B * C;
    if (ntiles > (1LL << 30)) return fail(0, "psgla_blur_grad: too many tiles");
    const dim3 grid((unsigned)ntiles);
    if (exact) {
        launch_blur<true>(a, l, grid, (hipStream_t)stream);
    } else if (!g_blur_no_sep && blur_rank1(a.hconv, K, a.sconv_r, a.sconv_c) &&
               blur_rank1(a.hcorr, K, a.scorr_r, a.scorr_c)) {
        launch_blur_sep(a, l, grid, (hipStream_t)stream);        // rank-1 taps: separable passes
    } else {
        launch_blur<false>(a, l, grid, (hipStream_t)stream);
    }
    return launch_check("blur_grad");
}

static AccArgs make_acc(const PsglaSchedule* s) {
    AccArgs a;
    a.n_inter = s->n_inter; a.nm = s->n_inter_mmse; a.coef = s->acc_coef;
    a.samples = s->samples; a.samples_cap = s->samples_cap;
    a.blocks = s->blocks; a.blocks2 = s->blocks2; a.blocks_cap = s->blocks_cap;
    a.d_step = (const long long*)s->d_step; a.off = s->step_offset;
    return a;
}

int psgla_relax_accumulate(const float* Y, const float* D, float* X, float alpha, int32_t alpha_is_one,
                           float* mean, float* sq, int32_t B, int64_t E, const PsglaSchedule* s, void* stream) {
    (void)alpha_is_one;
    if (!Y || !D || !X || !s || B <= 0 || E <= 0) return fail(0, "psgla_relax_accumulate: bad arguments");
    if (s->n_inter_mmse >= 0 && (!mean || !sq || !s->acc_coef)) return fail(0, "psgla_relax_accumulate: accumulators missing");
    const long long total = (long long)B * E;
    hipLaunchKernelGGL(relax_accumulate_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, Y,
                       D, X, alpha, B, (long long)E, mean, sq, make_acc(s));
    return launch_check("relax_accumulate");
}

int pnpula_update(const float* X, const float* gp, const float* gd, float* Xout, float delta, float lambd,
                  float brw, float c_min, float c_max, float* mean, float* sq, int32_t B, int64_t E,
                  uint64_t seed, int32_t chain0, const PsglaSchedule* s, void* stream) {
    if (!X || !gp || !gd || !Xout || !s || B <= 0 || E <= 0) return fail(0, "pnpula_update: bad arguments");
    if (s->n_inter_mmse >= 0 && (!mean || !sq || !s->acc_coef)) return fail(0, "pnpula_update: accumulators missing");
    const long long total = (long long)B * ((E + 3) / 4);
    if (B > 65535) return fail(0, "pnpula_update: more than 65535 chains in one launch");
    hipLaunchKernelGGL(pnpula_update_kernel, dim3(grid_chain(E / 4 + 1, B), B), dim3(256), 0, (hipStream_t)stream, X, gp,
                       gd, Xout, delta, lambd, brw, c_min, c_max, B, (long long)E, mean, sq,
                       (unsigned long long)seed, chain0, make_acc(s));
    return launch_check("pnpula_update");
}

int pnpula_prior_update(const float* X, const float* D, float alpha, float s2, const float* gd, const float* y,
                        int64_t y_chain_stride, const uint8_t* mask, int64_t mask_chain_stride, float sigma2, float* Xout,
                        float delta, float lambd, float brw, float c_min, float c_max, float* mean, float* sq, int32_t B,
                        int32_t C, int32_t H, int32_t W, uint64_t seed, int32_t chain0, const PsglaSchedule* s,
                        void* stream) {
    if (!X || !D || !Xout || !s || B <= 0 || C <= 0 || H <= 0 || W <= 0) return fail(0, "pnpula_prior_update: bad arguments");
    if (!gd && (!y || !mask)) return fail(0, "pnpula_prior_update: needs gd or the inpainting y / mask");
    if (s->n_inter_mmse >= 0 && (!mean || !sq || !s->acc_coef)) return fail(0, "pnpula_prior_update: accumulators missing");
    if (B > 65535) return fail(0, "pnpula_prior_update: more than 65535 chains in one launch");
    const long long HW = (long long)H * W, E = (long long)C * HW;
    hipLaunchKernelGGL(pnpula_prior_update_kernel, dim3(grid_chain(E / 4 + 1, B), B), dim3(256), 0, (hipStream_t)stream,
                       X, D, alpha, s2, gd, y, (long long)y_chain_stride, mask, (long long)mask_chain_stride, sigma2,
                       Xout, delta, lambd, brw, c_min, c_max, B, HW, E, mean, sq, (unsigned long long)seed, chain0,
                       make_acc(s));
    return launch_check("pnpula_prior_update");
}

int psgla_inpaint_grad(const float* X, const float* y, int64_t y_chain_stride, const uint8_t* mask,
                       int64_t mask_chain_stride, float* g, int32_t B, int32_t C, int32_t H, int32_t W, float sigma2,
                       void* stream) {
    if (!X || !y || !mask || !g || B <= 0 || C <= 0 || H <= 0 || W <= 0) return fail(0, "psgla_inpaint_grad: bad arguments");
    const long long total = (long long)B * C * H * W;
    if ((long long)B * C > 65535) return fail(0, "psgla_inpaint_grad: more than 65535 planes in one launch");
    hipLaunchKernelGGL(inpaint_grad_kernel, dim3(grid_chain((long long)H * W / 4 + 1, B * C), B * C), dim3(256), 0,
                       (hipStream_t)stream, X, y,
                       (long long)y_chain_stride, mask, (long long)mask_chain_stride, g, B, C, H, W, sigma2);
    return launch_check("inpaint_grad");
}

int psgla_relax_langevin_inpaint(const float* Y, const float* D, float* X, float alpha, int32_t alpha_is_one,
                                  const float* y, int64_t y_chain_stride, const uint8_t* mask,
                                  int64_t mask_chain_stride, float* Y_next, float* mean, float* sq, int32_t B,
                                  int32_t C, int32_t H, int32_t W, float sigma2, float c1, float c2, uint64_t seed,
                                  int32_t chain0, const PsglaSchedule* s, void* stream) {
    if (!D || !y || !mask || !Y_next || !s || B <= 0 || C <= 0 || H <= 0 || W <= 0)
        return fail(0, "psgla_relax_langevin_inpaint: bad arguments");
    if (!alpha_is_one && !Y) return fail(0, "psgla_relax_langevin_inpaint: Y required when alpha != 1");
    if (s->n_inter_mmse >= 0 && (!mean || !sq || !s->acc_coef))
        return fail(0, "psgla_relax_langevin_inpaint: accumulators missing");
    if ((long long)B * C > 65535) return fail(0, "psgla_relax_langevin_inpaint: more than 65535 planes in one launch");
    if (((long long)H * W) % 4 == 0)
        hipLaunchKernelGGL(relax_langevin_inpaint_kernel, dim3(grid_chain((long long)H * W / 4 + 1, B * C), B * C),
                           dim3(256), 0, (hipStream_t)stream, Y, D, X, alpha, (int)(alpha_is_one != 0), y,
                           (long long)y_chain_stride, mask, (long long)mask_chain_stride, Y_next, B, C, H, W, sigma2,
                           c1, c2, (unsigned long long)seed, chain0, mean, sq, make_acc(s));
    else
        hipLaunchKernelGGL(relax_langevin_inpaint_any_kernel,
                           dim3(grid_chain(((long long)C * H * W + 3) / 4, B), B), dim3(256), 0, (hipStream_t)stream,
                           Y, D, X, alpha, (int)(alpha_is_one != 0), y, (long long)y_chain_stride, mask,
                           (long long)mask_chain_stride, Y_next, B, C, H, W, sigma2, c1, c2,
                           (unsigned long long)seed, chain0, mean, sq, make_acc(s));
    return launch_check("relax_langevin_inpaint");
}

int psgla_debug_bm_tables(float* r, float* cs, float* sn, uint32_t k0, uint32_t n, void* stream) {
    if (!r || !cs || !sn) return fail(0, "psgla_debug_bm_tables: null");
    hipLaunchKernelGGL(bm_tables_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, r, cs, sn, k0, n);
    return launch_check("bm_tables");
}

int psgla_bias_act(float* y, const float* bias, int64_t n, int32_t C, int64_t hw, int32_t relu, void* stream) {
    if (!y || !bias || n < 0 || C <= 0 || hw < 0) return fail(0, "psgla_bias_act: bad arguments");
    if (n % 4 != 0) return fail(0, "psgla_bias_act: element count must be a multiple of 4");
    if (hw == 0 && C % 4 != 0) return fail(0, "psgla_bias_act: NHWC needs C % 4 == 0");
    if (hw > 0 && hw % 4 != 0) return fail(0, "psgla_bias_act: NCHW needs H*W % 4 == 0");
    if (n == 0) return 0;
    const long long n4 = n / 4;
    const long long grid = (n4 + 255) / 256 < 256LL * 32 ? (n4 + 255) / 256 : 256LL * 32;
    hipLaunchKernelGGL(bias_act_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, y, bias, n4, C,
                       (long long)hw, relu);
    return launch_check("bias_act");
}

int psgla_advance_step(int64_t* d_step, void* stream) {
    if (!d_step) return fail(0, "psgla_advance_step: null");
    hipLaunchKernelGGL(advance_step_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, (long long*)d_step);
    return launch_check("advance_step");
}

}  // extern "C"
