// Band kernel (tv_main_kernel) + finaliser (tv_finalise_kernel): the temporally blocked PSGLA + TV step for
// shapes the row stream does not take, and the standalone TV prox (psgla_tv_prox).
// (library overview: psgla_common.hpp)
#include "psgla_common.hpp"

namespace psgla {

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
                // psgla noise v2: the lane's 4 columns (gj0 a multiple of 4) are one quad of the row
                normal_quad(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step, TAG_LANGEVIN,
                            noise_quad((size_t)c * H + gi[r], gj0, W), Z);
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
                } else {
#pragma unroll
                    for (int k = 0; k < CPL; ++k) {
                        const bool ok = colok[k];
                        X[k] = ok ? xin[base + k] : 0.f;
                        yo[k] = ok ? yb[k] : 0.f;
                        mk[k] = ok ? (float)mb[k] : 0.f;
                        Z[k] = ok ? Z[k] : 0.f;
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
                    xv = __builtin_fmaf(TV_TAU, f4get(yrow, k) - t, xo) * TV_INV_OPT;
                    zv = __builtin_fmaf(2.0f, xv, -xo);
                    xn = __builtin_fmaf(TV_RHO, xv - xo, xo);
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
                    const float v0 = __builtin_fmaf(TV_SIG, g0, uo0);
                    const float v1 = __builtin_fmaf(TV_SIG, g1, uo1);
                    const float s2 = __builtin_fmaf(v0, v0, v1 * v1);
                    const float f = tv_proj_factor(vconst(a.ths), s2);
                    u0[r][k] = __builtin_fmaf(TV_RHO, __builtin_fmaf(v0, f, -uo0), uo0);
                    u1[r][k] = __builtin_fmaf(TV_RHO, __builtin_fmaf(v1, f, -uo1), uo1);
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

template <bool EXACT, int FRONT, bool ALPHA1>
void launch_band_main(const TvArgs& a, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((tv_main_kernel<EXACT, FRONT, ALPHA1>), grid, dim3(TV_THREADS), 0, st, a);
}
template <bool EXACT, int FRONT, bool ALPHA1>
void launch_band_finalise(const TvArgs& a, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((tv_finalise_kernel<EXACT, FRONT, ALPHA1>), grid, dim3(TV_THREADS), 0, st, a);
}
#define PSGLA_BAND(E, F, A) \
    template void launch_band_main<E, F, A>(const TvArgs&, dim3, hipStream_t); \
    template void launch_band_finalise<E, F, A>(const TvArgs&, dim3, hipStream_t);
PSGLA_BAND(true, FRONT_INPAINT, true) PSGLA_BAND(true, FRONT_INPAINT, false) PSGLA_BAND(true, FRONT_GIVEN, true)
PSGLA_BAND(false, FRONT_INPAINT, true) PSGLA_BAND(false, FRONT_INPAINT, false) PSGLA_BAND(false, FRONT_GIVEN, true)
#undef PSGLA_BAND

}  // namespace psgla
