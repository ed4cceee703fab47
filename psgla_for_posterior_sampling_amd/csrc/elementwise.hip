// Generic elementwise kernels (opaque closures, DnCNN / DRUNet engines, PnP-ULA) and their C ABI entry points.
// (library overview: psgla_common.hpp)
#include "psgla_common.hpp"

namespace psgla {

// ---------------------------------------------------------------------------------------
// Generic elementwise kernels (opaque closures; also the first / last steps of fused paths)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ long long read_step(const long long* d, long long off) {
    return (d ? *d : 0LL) + off;
}

// psgla noise v2 over a chain of E elements in rows of W (noise.hpp): quads never straddle two rows, so quad q
// covers the chain's elements [e, e + n), e = (q / QW) W + 4 (q % QW), n = min(4, W - 4 (q % QW)), QW =
// ceil(W / 4); (E / W) QW quads per chain.  W % 4 == 0: e = 4 q, n = 4 (no division).
__device__ __forceinline__ long long quad_span(long long q, int W, int QW, int& n) {
    if ((W & 3) == 0) {
        n = 4;
        return q << 2;
    }
    const long long row = q / QW;
    const int k = (int)(q - row * QW);
    n = min(4, W - 4 * k);
    return row * W + 4 * k;
}

__global__ void normal_fill_kernel(float* out, int B, long long E, int W, unsigned long long seed, int chain0,
                                   const long long* d_step, long long off, uint32_t tag) {
    const long long step = read_step(d_step, off);
    const int QW = (W + 3) >> 2;
    const long long Q = (E / W) * QW;
    const long long total = (long long)B * Q;
    for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
         t += (long long)gridDim.x * blockDim.x) {
        const int b = (int)(t / Q);
        const long long q = t - (long long)b * Q;
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)step, tag, (uint32_t)q, z);
        int n;
        const long long e = quad_span(q, W, QW, n);
        float* o = out + (size_t)b * E + e;
        if ((W & 3) == 0) {
            *reinterpret_cast<float4*>(o) = make_float4(z[0], z[1], z[2], z[3]);
        } else {
            for (int j = 0; j < n; ++j) o[j] = z[j];
        }
    }
}

// Y = (X + c1 g) + c2 Z   (restoration_algorithms.py:236)
__global__ void langevin_update_kernel(const float* X, const float* g, float* Y, int B, long long E, int W,
                                       float c1, float c2, unsigned long long seed, int chain0,
                                       const long long* d_step, long long off) {
    // grid: (noise quads of a chain, chain)
    const long long step = read_step(d_step, off);
    const int QW = (W + 3) >> 2;
    const long long Q = (E / W) * QW;
    const int b = blockIdx.y;
    const bool vec = (W & 3) == 0;
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < Q;
         q += (long long)gridDim.x * blockDim.x) {
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)step, TAG_LANGEVIN, (uint32_t)q, z);
        int n;
        const size_t i0 = (size_t)b * E + (size_t)quad_span(q, W, QW, n);
        if (vec) {
            const float4 x = ld4(X + i0), gg = ld4(g + i0);
            st4(Y + i0, (x.x + c1 * gg.x) + c2 * z[0], (x.y + c1 * gg.y) + c2 * z[1],
                (x.z + c1 * gg.z) + c2 * z[2], (x.w + c1 * gg.w) + c2 * z[3]);
        } else {
            for (int j = 0; j < n; ++j) Y[i0 + j] = (X[i0 + j] + c1 * g[i0 + j]) + c2 * z[j];
        }
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

// The same pass for W % 4 != 0 (set1c / CBSD68 are 481 x 321): one thread per noise quad of the chain (row-aligned,
// psgla noise v2), scalar loads.  grid: (noise quads of a chain, chain)
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
    const int QW = (W + 3) >> 2;
    const long long Q = (long long)C * H * QW;
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < Q; q += (long long)gridDim.x * blockDim.x) {
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)(step + 1), TAG_LANGEVIN, (uint32_t)q, z);
        int n;
        const long long e0 = quad_span(q, W, QW, n);
        const long long m0 = e0 % HW;                      // a quad lies in one row, so in one plane
        for (int j = 0; j < n; ++j) {
            const long long e = e0 + j;
            const size_t idx = (size_t)b * E + e;
            const float x = alpha1 ? D[idx] : (1.0f - alpha) * Y[idx] + alpha * D[idx];
            if (X_out) X_out[idx] = x;
            acc_elem(s, step, idx, BE, x, mean, sq);
            const float m = (float)mp[m0 + j];
            const float g = (-m * (x - yp[e])) / sigma2;
            Y_next[idx] = (x + c1 * g) + c2 * z[j];
        }
    }
}

// PnP-ULA (restoration_algorithms.py:104-115)
__global__ void pnpula_update_kernel(const float* X, const float* gp, const float* gd, float* Xo,
                                     float delta, float lambd, float brw, float cmin, float cmax, int B,
                                     long long E, int W, float* mean, float* sq, unsigned long long seed,
                                     int chain0, AccArgs s) {
    // grid: (noise quads of a chain, chain)
    const long long step = read_step(s.d_step, s.off);
    const int QW = (W + 3) >> 2;
    const long long Q = (E / W) * QW;
    const size_t BE = (size_t)B * E;
    const int b = blockIdx.y;
    const bool vec = (W & 3) == 0;
    const AccStep st = acc_step(s, step, mean);
    for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < Q;
         q += (long long)gridDim.x * blockDim.x) {
        float z[4];
        normal_quad(seed, (uint32_t)(chain0 + b), (uint32_t)step, TAG_LANGEVIN, (uint32_t)q, z);
        int n;
        const size_t i0 = (size_t)b * E + (size_t)quad_span(q, W, QW, n);
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
            for (int j = 0; j < n; ++j) {
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
// pnpula_update.  grid: (noise quads of a chain, chain): row-aligned quads (psgla noise v2).
__global__ void pnpula_prior_update_kernel(const float* X, const float* D, float alpha, float s2, const float* gd,
                                           const float* y, long long y_cs, const uint8_t* mask, long long m_cs,
                                           float sigma2, float* Xo, float delta, float lambd, float brw, float cmin,
                                           float cmax, int B, long long HW, long long E, int W, float* mean,
                                           float* sq, unsigned long long seed, int chain0, AccArgs s) {
    const long long step = read_step(s.d_step, s.off);
    const int QW = (W + 3) >> 2;
    const long long Q = (E / W) * QW;
    const size_t BE = (size_t)B * E;
    const int b = blockIdx.y;
    const bool vec = (W & 3) == 0;
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
        int n;
        const long long e0 = quad_span(q, W, QW, n);
        const size_t i0 = (size_t)b * E + (size_t)e0;
        if (vec) {
            const float4 x = ld4(X + i0), d = ld4(D + i0);
            float g[4];
            if (gd) {
                const float4 g4 = ld4(gd + i0);
                g[0] = g4.x; g[1] = g4.y; g[2] = g4.z; g[3] = g4.w;
            } else {
                const long long e = e0;
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
            for (int j = 0; j < n; ++j) {
                const long long e = e0 + j;
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

using namespace psgla;

extern "C" {

int psgla_normal_fill(float* out, int32_t B, int64_t E, int32_t W, uint64_t seed, int32_t chain0, const int64_t* d_step,
                      int64_t step_offset, uint32_t tag, void* stream) {
    if (!out || B <= 0 || E <= 0 || W <= 0 || E % W != 0) return fail(0, "psgla_normal_fill: bad arguments");
    const long long total = (long long)B * (E / W) * ((W + 3) / 4);
    hipLaunchKernelGGL(normal_fill_kernel, dim3(grid_for(total, 256)), dim3(256), 0, (hipStream_t)stream, out, B,
                       (long long)E, (int)W, (unsigned long long)seed, chain0, (const long long*)d_step,
                       (long long)step_offset, tag);
    return launch_check("normal_fill");
}

int psgla_langevin_update(const float* X, const float* g, float* Y, int32_t B, int64_t E, int32_t W, float c1,
                          float c2, uint64_t seed, int32_t chain0, const int64_t* d_step, int64_t step_offset,
                          void* stream) {
    if (!X || !g || !Y || B <= 0 || E <= 0 || W <= 0 || E % W != 0) return fail(0, "psgla_langevin_update: bad arguments");
    if (B > 65535) return fail(0, "psgla_langevin_update: more than 65535 chains in one launch");
    const long long Q = (E / W) * ((W + 3) / 4);
    hipLaunchKernelGGL(langevin_update_kernel, dim3(grid_chain(Q, B), B), dim3(256), 0, (hipStream_t)stream, X,
                       g, Y, B, (long long)E, (int)W, c1, c2, (unsigned long long)seed, chain0,
                       (const long long*)d_step, (long long)step_offset);
    return launch_check("langevin_update");
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
                  float brw, float c_min, float c_max, float* mean, float* sq, int32_t B, int64_t E, int32_t W,
                  uint64_t seed, int32_t chain0, const PsglaSchedule* s, void* stream) {
    if (!X || !gp || !gd || !Xout || !s || B <= 0 || E <= 0 || W <= 0 || E % W != 0)
        return fail(0, "pnpula_update: bad arguments");
    if (s->n_inter_mmse >= 0 && (!mean || !sq || !s->acc_coef)) return fail(0, "pnpula_update: accumulators missing");
    if (B > 65535) return fail(0, "pnpula_update: more than 65535 chains in one launch");
    const long long Q = (E / W) * ((W + 3) / 4);
    hipLaunchKernelGGL(pnpula_update_kernel, dim3(grid_chain(Q, B), B), dim3(256), 0, (hipStream_t)stream, X, gp,
                       gd, Xout, delta, lambd, brw, c_min, c_max, B, (long long)E, (int)W, mean, sq,
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
    const long long Q = (long long)C * H * ((W + 3) / 4);
    hipLaunchKernelGGL(pnpula_prior_update_kernel, dim3(grid_chain(Q, B), B), dim3(256), 0, (hipStream_t)stream,
                       X, D, alpha, s2, gd, y, (long long)y_chain_stride, mask, (long long)mask_chain_stride, sigma2,
                       Xout, delta, lambd, brw, c_min, c_max, B, HW, E, (int)W, mean, sq, (unsigned long long)seed, chain0,
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
    if (W % 4 == 0)   // the vector pass's plane-linear quads are the noise quads only for W % 4 == 0
        hipLaunchKernelGGL(relax_langevin_inpaint_kernel, dim3(grid_chain((long long)H * W / 4 + 1, B * C), B * C),
                           dim3(256), 0, (hipStream_t)stream, Y, D, X, alpha, (int)(alpha_is_one != 0), y,
                           (long long)y_chain_stride, mask, (long long)mask_chain_stride, Y_next, B, C, H, W, sigma2,
                           c1, c2, (unsigned long long)seed, chain0, mean, sq, make_acc(s));
    else
        hipLaunchKernelGGL(relax_langevin_inpaint_any_kernel,
                           dim3(grid_chain((long long)C * H * ((W + 3) / 4), B), B), dim3(256), 0, (hipStream_t)stream,
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
