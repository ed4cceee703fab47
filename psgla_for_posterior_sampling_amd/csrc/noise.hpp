// In-register Gaussian noise for the Langevin step (replaces torch.randn at
// /root/reference/restoration_algorithms.py:232 (psgla) and :104 (pnpula)).
//
// "psgla noise v2": counter-based, so any element of any chain at any step can be
// regenerated anywhere (tiles recompute their halo's noise instead of reading it):
//   ctr = {quad, step, tag, seed_hi}, key = {seed_lo, chain}
//   Philox4x32-10 -> 4 x u32 -> two Box-Muller pairs -> 4 x N(0,1) fp32
//   a chain's C*H*W image is C*H rows of W elements; element (row, col) uses output
//   (col & 3) of quad row * ceil(W/4) + (col >> 2): a quad never straddles two rows, so
//   a lane holding 4 columns of a row (from a multiple of 4) needs exactly one Philox for
//   any W.  For W % 4 == 0 this is quad e >> 2, output e & 3 of the flat index e (the
//   "v1" stream of rounds 1-3, which numbered quads over the flat index for every W and
//   made W % 4 != 0 rows straddle two quads).
// log / sin / cos are fixed fp32 polynomials evaluated with explicit fmaf and the
// square root is IEEE-rounded (sqrtf under the default -fhip-fp32-correctly-rounded-divide-sqrt;
// NB: HIP's __fsqrt_rn is the native approximation), so the stream is bit-identical to the
// CPU checker's (oracle/noise.c); tests/test_gpu_parity.py checks all 2^24 radii
// and all 2^24 angles exhaustively.  Compile with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psgla {

__device__ __forceinline__ void philox4x32_10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0;
        const uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

// log(u), u in (0,1]: u = 2^e m with m in [sqrt(1/2), sqrt(2)); log1p(f) = f + f^2 P(f), f = m-1.
__device__ __forceinline__ float log_unit(float u) {
    uint32_t bits = __float_as_uint(u);
    int e = (int)(bits >> 23) - 127;
    uint32_t mb = (bits & 0x007FFFFFu) | 0x3F800000u;
    const bool hi = mb > 0x3FB504F3u;
    mb = hi ? mb - 0x00800000u : mb;
    e = hi ? e + 1 : e;
    const float f = __uint_as_float(mb) - 1.0f;
    float p = -0.07866667956113815f;
    p = __builtin_fmaf(p, f, 0.12821748852729797f);
    p = __builtin_fmaf(p, f, -0.131016343832016f);
    p = __builtin_fmaf(p, f, 0.1418900042772293f);
    p = __builtin_fmaf(p, f, -0.1662759929895401f);
    p = __builtin_fmaf(p, f, 0.2000196874141693f);
    p = __builtin_fmaf(p, f, -0.2500077188014984f);
    p = __builtin_fmaf(p, f, 0.33333322405815125f);
    p = __builtin_fmaf(p, f, -0.4999999701976776f);
    const float ff = f * f;
    const float l1p = __builtin_fmaf(ff, p, f);
    const float fe = (float)e;
    return __builtin_fmaf(fe, 0.693145751953125f, __builtin_fmaf(fe, 1.428606765330187e-06f, l1p));
}

// r = sqrt(-2 log u), u = (k24 + 1) 2^-24
__device__ __forceinline__ float bm_radius(uint32_t k24) {
    const float u = (float)(k24 + 1u) * 5.9604644775390625e-08f;
    return sqrtf(-2.0f * log_unit(u));
}

// (cos, sin)(2 pi k24 2^-24): nearest quarter turn n, remainder f in [-1/2, 1/2] quarter turns.
__device__ __forceinline__ void bm_angle(uint32_t k24, float& cs, float& sn) {
    const uint32_t n = (k24 + (1u << 21)) >> 22;
    const int32_t rem = (int32_t)k24 - (int32_t)(n << 22);
    const float f = (float)rem * 2.384185791015625e-07f;
    const float w = f * f;
    float s = 0.00015820653061382473f;
    s = __builtin_fmaf(s, w, -0.004681266378611326f);
    s = __builtin_fmaf(s, w, 0.07969257980585098f);
    s = __builtin_fmaf(s, w, -0.6459640860557556f);
    s = __builtin_fmaf(s, w, 1.5707963705062866f);
    s = s * f;
    float c = -2.4850989575497806e-05f;
    c = __builtin_fmaf(c, w, 0.000919161771889776f);
    c = __builtin_fmaf(c, w, -0.020863467827439308f);
    c = __builtin_fmaf(c, w, 0.25366950035095215f);
    c = __builtin_fmaf(c, w, -1.2337005138397217f);
    c = __builtin_fmaf(c, w, 1.0f);
    // rotate by n quarter turns: odd n swaps (c,s)->(-s,c); n&2 negates both
    const bool odd = (n & 1u) != 0u;
    float a = odd ? -s : c;
    float b = odd ? c : s;
    const bool neg = (n & 2u) != 0u;
    cs = neg ? -a : a;
    sn = neg ? -b : b;
}

__device__ __forceinline__ void box_muller(uint32_t x0, uint32_t x1, float& z0, float& z1) {
    const float r = bm_radius(x0 >> 8);
    float c, s;
    bm_angle(x1 >> 8, c, s);
    z0 = r * c;
    z1 = r * s;
}

__device__ __forceinline__ void normal_quad(uint64_t seed, uint32_t chain, uint32_t step, uint32_t tag,
                                            uint32_t quad, float z[4]) {
    uint32_t c0 = quad, c1 = step, c2 = tag, c3 = (uint32_t)(seed >> 32);
    philox4x32_10(c0, c1, c2, c3, (uint32_t)seed, chain);
    box_muller(c0, c1, z[0], z[1]);
    box_muller(c2, c3, z[2], z[3]);
}

// the quad holding element (row, col) of a chain's image of W-element rows
__device__ __forceinline__ uint32_t noise_quad(size_t row, int col, int W) {
    return (uint32_t)(row * (size_t)((W + 3) >> 2) + (size_t)(col >> 2));
}

}  // namespace psgla
