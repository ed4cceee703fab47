/*
 * oracle/noise.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * CPU restatement of the Langevin noise stream that the HIP kernels generate
 * in registers.  It replaces `torch.randn(im_shape, generator=gen)` of
 *   /root/reference/restoration_algorithms.py:232   (psgla)
 *   /root/reference/restoration_algorithms.py:104   (pnpula)
 * The reference draws from torch's generator; that stream depends on the
 * device (CPU mt19937 vs CUDA Philox with a device-dependent thread mapping),
 * so parity is defined on an *injected* common stream: the golden fixtures
 * are produced by the reference's own psgla/pnpula with torch.randn patched
 * to return this stream (tests/golden/make_golden.py).
 *
 * Stream definition ("psgla noise v2"), written independently of the HIP
 * implementation in psgla_for_posterior_sampling_amd/csrc/noise.hpp:
 *   ctr = {quad, step, tag, seed_hi}, key = {seed_lo, chain}
 *   x[0..3] = Philox4x32-10(ctr, key)   (Salmon et al., SC'11; Random123)
 *   (z0,z1) = BoxMuller(x0,x1), (z2,z3) = BoxMuller(x2,x3)
 *   a chain's C*H*W image is C*H rows of W elements; element (row, col) at
 *   Langevin step i takes z[col & 3] of quad row * ceil(W/4) + (col >> 2):
 *   quads never straddle two rows.  For W % 4 == 0 that is z[e & 3] of quad
 *   e >> 2 for the flat index e = row * W + col (the round-1..3 "v1" stream,
 *   which numbered quads over the flat index for every W).
 *   BoxMuller(a,b): u = ((a>>8)+1)*2^-24 in (0,1];  r = sqrt(-2 log u);
 *     theta = 2*pi*(b>>8)*2^-24;  (r cos theta, r sin theta)
 *   log/sin/cos are fixed fp32 polynomials evaluated with explicit fmaf, and
 *   sqrt is IEEE correctly rounded, so the CPU and GPU streams are
 *   bit-identical (checked exhaustively in tests/test_gpu_noise.py).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

static inline uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t *hi) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, hi1;
        uint32_t lo0 = mulhilo(PHILOX_M0, c0, &hi0);
        uint32_t lo1 = mulhilo(PHILOX_M1, c2, &hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += PHILOX_W0; k1 += PHILOX_W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static inline float as_float(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t as_uint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* log(u) for u in (0,1]: u = 2^e * m, m in [sqrt(.5), sqrt(2)); log1p(m-1) = f + f^2 P(f). */
static const float LOG_P[9] = {
    -0.4999999701976776f, 0.33333322405815125f, -0.2500077188014984f, 0.2000196874141693f,
    -0.1662759929895401f, 0.1418900042772293f, -0.131016343832016f, 0.12821748852729797f,
    -0.07866667956113815f};
static const float LN2_HI = 0.693145751953125f;   /* 0x3F317200 */
static const float LN2_LO = 1.428606765330187e-06f;

float oracle_logf_unit(float u) {
    uint32_t bits = as_uint(u);
    int e = (int)(bits >> 23) - 127;
    uint32_t mb = (bits & 0x007FFFFFu) | 0x3F800000u;
    if (mb > 0x3FB504F3u) { mb -= 0x00800000u; e += 1; }
    float f = as_float(mb) - 1.0f;
    float p = LOG_P[8];
    for (int k = 7; k >= 0; --k) p = fmaf(p, f, LOG_P[k]);
    float ff = f * f;
    float l1p = fmaf(ff, p, f);
    float fe = (float)e;
    return fmaf(fe, LN2_HI, fmaf(fe, LN2_LO, l1p));
}

/* sin(pi/2 f) = f S(f^2), cos(pi/2 f) = C(f^2) for f in [-1/2, 1/2]. */
static const float SIN_S[5] = {1.5707963705062866f, -0.6459640860557556f, 0.07969257980585098f,
                               -0.004681266378611326f, 0.00015820653061382473f};
static const float COS_C[6] = {1.0f, -1.2337005138397217f, 0.25366950035095215f,
                               -0.020863467827439308f, 0.000919161771889776f,
                               -2.4850989575497806e-05f};

/* radius r(a) = sqrt(-2 log u(a)) for the 24-bit index k = a >> 8 */
float oracle_bm_radius(uint32_t k24) {
    float u = (float)(k24 + 1u) * 5.9604644775390625e-08f; /* 2^-24 */
    float l = oracle_logf_unit(u);
    return sqrtf(-2.0f * l);
}

/* (cos, sin) of 2*pi*k*2^-24 for the 24-bit index k = b >> 8 */
void oracle_bm_angle(uint32_t k24, float *c_out, float *s_out) {
    uint32_t n = (k24 + (1u << 21)) >> 22;               /* nearest quarter turn, 0..4 */
    int32_t rem = (int32_t)k24 - (int32_t)(n << 22);     /* in [-2^21, 2^21] */
    float f = (float)rem * 2.384185791015625e-07f;       /* 2^-22, exact */
    float w = f * f;
    float s = SIN_S[4];
    for (int k = 3; k >= 0; --k) s = fmaf(s, w, SIN_S[k]);
    s = s * f;
    float c = COS_C[5];
    for (int k = 4; k >= 0; --k) c = fmaf(c, w, COS_C[k]);
    float cs, sn;
    switch (n & 3u) {
        case 0: cs = c; sn = s; break;
        case 1: cs = -s; sn = c; break;
        case 2: cs = -c; sn = -s; break;
        default: cs = s; sn = -c; break;
    }
    *c_out = cs; *s_out = sn;
}

static inline void box_muller(uint32_t a, uint32_t b, float *z0, float *z1) {
    float r = oracle_bm_radius(a >> 8);
    float c, s;
    oracle_bm_angle(b >> 8, &c, &s);
    *z0 = r * c;
    *z1 = r * s;
}

void oracle_normal_quad(uint64_t seed, uint32_t chain, uint32_t step, uint32_t tag,
                        uint32_t quad, float z[4]) {
    uint32_t ctr[4] = {quad, step, tag, (uint32_t)(seed >> 32)};
    uint32_t key[2] = {(uint32_t)seed, chain};
    uint32_t x[4];
    oracle_philox4x32_10(ctr, key, x);
    box_muller(x[0], x[1], &z[0], &z[1]);
    box_muller(x[2], x[3], &z[2], &z[3]);
}

/* Fill one chain's image of `rows` rows of W elements at one step (row-aligned quads, see above). */
void oracle_normal_fill_rows(float *out, uint64_t rows, uint32_t W, uint64_t seed, uint32_t chain,
                             uint32_t step, uint32_t tag) {
    float z[4];
    const uint64_t qw = ((uint64_t)W + 3) >> 2;        /* quads per row */
    for (uint64_t r = 0; r < rows; ++r) {
        for (uint64_t k = 0; k < qw; ++k) {
            oracle_normal_quad(seed, chain, step, tag, (uint32_t)(r * qw + k), z);
            for (uint32_t j = 0; j < 4; ++j) {
                const uint64_t col = 4 * k + j;
                if (col < W) out[r * W + col] = z[j];
            }
        }
    }
}

/* Exhaustive tables for the GPU bit-exactness test (2^24 entries each). */
void oracle_radius_table(float *out, uint32_t k_begin, uint32_t count) {
    for (uint32_t i = 0; i < count; ++i) out[i] = oracle_bm_radius(k_begin + i);
}
void oracle_angle_table(float *cos_out, float *sin_out, uint32_t k_begin, uint32_t count) {
    for (uint32_t i = 0; i < count; ++i) oracle_bm_angle(k_begin + i, &cos_out[i], &sin_out[i]);
}
