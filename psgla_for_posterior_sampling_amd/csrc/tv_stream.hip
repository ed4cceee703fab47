// Row-streaming PSGLA + TV step (tv_stream_kernel): the 64-chain production kernel.
// (library overview: psgla_common.hpp)
#include "psgla_common.hpp"

namespace psgla {


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


// LDS of a workgroup.  Rings hold (x2, u2) rows between stages, u2 in its memory layout: two float4 per lane,
// (u0, u1) of the lane's columns 0-1 (ua) and 2-3 (ub).  A1 (alpha == 1, the benched case): stage 1 reads its
// TV input (x2 = X, u2) straight from the front's LDS-DMA staging -- no ring 0 copy by the front -- so those
// staging parts are triple-buffered (a row's slot is re-targeted by the DMA of the row 12 later, issued after
// stage 1 has read it); the observation y and the mask stay double-buffered (only the front reads them).
// !A1: the front's staging (X, y, u2 lo / hi, x2) is double-buffered and the front writes ring 0.
template <bool A1>
struct StreamSharedT {
    static constexpr int NR = SP_MAXST + (A1 ? 0 : 1);   // rings: stage outputs (+ ring 0 = the front's, !A1)
    float4 x2[NR][2][WAVE];
    float4 ua[NR][2][WAVE];
    float4 ub[NR][2][WAVE];
    float4 y[SP_YRING][WAVE];             // Y rows (prox anchor), alive from the front to the back
    // LDS-DMA staging (global_load_lds_dwordx4): a front wave's next rows and a back wave's next mean / sq rows
    // land here without occupying VGPRs.  A1: fsx[fw][row slot (q / 4) % 3][X, u2 lo, u2 hi], fsy[fw][(q / 4) % 2]
    // = y; !A1: fsx[fw][(q / 4) % 2][X, y, u2 lo, u2 hi, x2].
    float4 fsx[SP_FRONT][A1 ? 3 : 2][A1 ? 3 : 5][WAVE];
    float4 fsy[SP_FRONT][A1 ? 2 : 1][WAVE];
    uint32_t fmk[SP_FRONT][2][WAVE];
    float4 bst[SP_BACK][2][2][WAVE];
    float red[SP_MAXSEG][2][SP_MAXST][2];   // rel-err partial sums per (stream segment, half-wave, iteration)
    // ring holding the output of stage k (k = 0: the front's ring 0, !A1 only)
    static __device__ __forceinline__ constexpr int rk(int k) { return A1 ? k - 1 : k; }
    __device__ __forceinline__ float4* stX(int fw, int q) { return A1 ? &fsx[fw][((q >> 2) % 3)][0][0] : &fsx[fw][(q >> 2) & 1][0][0]; }
    __device__ __forceinline__ float4* stY(int fw, int q) { return A1 ? &fsy[fw][(q >> 2) & 1][0] : &fsx[fw][(q >> 2) & 1][1][0]; }
    __device__ __forceinline__ float4* stUa(int fw, int q) { return A1 ? &fsx[fw][((q >> 2) % 3)][1][0] : &fsx[fw][(q >> 2) & 1][2][0]; }
    __device__ __forceinline__ float4* stUb(int fw, int q) { return A1 ? &fsx[fw][((q >> 2) % 3)][2][0] : &fsx[fw][(q >> 2) & 1][3][0]; }
    __device__ __forceinline__ float4* stX2(int fw, int q) { return &fsx[fw][(q >> 2) & 1][A1 ? 0 : 4][0]; }
};


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
        m.pl0 = wg;                   // virtual plane (plane * st_nsegs + column segment, or a pair of them)
        return;
    }
    const long long T = (long long)a.st_nvp * H;
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

// Column geometry of a virtual plane: the real plane, the start of the segment's wave window (f0) and its core
// columns [cc0, cc1).  Without GEN there is one segment (vp = plane, the whole row).  GEN: vp = item = plane *
// st_nsegs + column segment, a 256-column window.  HALF (st_half): vp is a PAIR of items, 2 vp + h in half-wave h
// (lanes 32 h .. 32 h + 31, a 128-column window each); a pair's missing second item (odd item count) repeats the
// first in a disabled half (on = false: nothing stored or counted there); vp >= st_nvp -- the early-stop
// recompute -- is item vp - st_nvp in both halves.  h: the lane's half (HALF only, per lane).
struct SegGeo {
    int rp, f0, cc0, cc1;
    bool on;
};
template <bool GEN, bool HALF = false>
__device__ __forceinline__ SegGeo seg_geo(const TvArgs& a, int vp, int h = 0) {
    SegGeo g;
    g.on = true;
    if (!GEN) {
        g.rp = vp; g.f0 = 0; g.cc0 = 0; g.cc1 = a.W;
        return g;
    }
    int item = vp;
    if (HALF) {
        const int nitems = a.B * a.C * a.st_nsegs;
        if (vp >= a.st_nvp) {
            item = vp - a.st_nvp;
        } else {
            item = 2 * vp + h;
            if (item >= nitems) { item = 2 * vp; g.on = false; }
        }
    }
    const int ns = a.st_nsegs;
    g.rp = item / ns;
    const int sgi = item - g.rp * ns;
    g.cc0 = sgi * a.st_seg_w;
    g.cc1 = (sgi == ns - 1) ? a.W : min(a.W, g.cc0 + a.st_seg_w);   // the last segment takes the rest
    g.f0 = max(0, g.cc0 - a.st_halo) & ~3;
    return g;
}
// a lane's position in its window: HALF windows are half-waves
template <bool HALF>
__device__ __forceinline__ int lcol(int lane) { return HALF ? (lane & 31) : lane; }

// Position of a role's current row in the stream; advanced monotonically (the segment walk
// runs only when a plane boundary is crossed).
// The cursor also caches its segment's address geometry (plane / observation / mask bases, chain, noise
// element base, GEN: the wave window's first column), recomputed only when the cursor enters a new segment:
// the per-row address and noise-counter arithmetic of the front and back roles is then adds and one
// multiply, with no integer division on their per-step paths.
struct RowGeo {
    size_t pbase;       // element offset of the (real) plane in the (B, C, H, ldw) state buffers
    size_t ybase;       // element offset of the plane in the observation (chain stride y_cs)
    size_t mbase;       // byte offset of the chain's mask (chain stride m_cs)
    size_t rbase;       // the plane's first row among its chain's C*H rows (noise counter, psgla noise v2)
    int bb;             // chain (batch entry)
    int f0;             // first column of the wave window (GEN; 0 otherwise)
    int cc0, cc1;       // core columns of the segment
    bool on;            // HALF: the lane's half-window holds an item
};
struct RowCursor {
    int q, s, p, r, qend;
    RowGeo g;
};
template <bool GEN, bool HALF>
__device__ __forceinline__ RowGeo row_geo(const TvArgs& a, int vp) {
    const SegGeo sg = seg_geo<GEN, HALF>(a, vp, HALF ? (int)((threadIdx.x & 63) >> 5) : 0);
    const size_t HW = (size_t)a.H * a.ldw;
    RowGeo g;
    g.bb = sg.rp / a.C;
    const int cc = sg.rp - g.bb * a.C;
    g.pbase = (size_t)sg.rp * HW;
    g.ybase = (size_t)g.bb * a.y_cs + (size_t)cc * HW;
    g.mbase = (size_t)g.bb * a.m_cs;
    g.rbase = (size_t)cc * a.H;
    g.f0 = sg.f0;
    g.cc0 = sg.cc0;
    g.cc1 = sg.cc1;
    g.on = sg.on;
    return g;
}
template <bool GEN, bool HALF>
__device__ __forceinline__ void cursor_seek(const TvArgs& a, const RowMap& m, RowCursor& c) {
    while (c.s + 1 < m.ns && c.q >= m.qs(c.s + 1)) ++c.s;
    c.qend = m.qs(c.s + 1);
    c.p = m.pl(c.s);
    c.r = m.lo(c.s) + (c.q - m.qs(c.s));
    c.g = row_geo<GEN, HALF>(a, c.p);
}
template <bool GEN, bool HALF>
__device__ __forceinline__ void cursor_init(const TvArgs& a, const RowMap& m, RowCursor& c, int q) {
    c.q = q; c.s = 0;
    cursor_seek<GEN, HALF>(a, m, c);
}
template <bool GEN, bool HALF>
__device__ __forceinline__ void cursor_advance(const TvArgs& a, const RowMap& m, RowCursor& c, int d) {
    c.q += d; c.r += d;
    if (c.q >= c.qend && c.s + 1 < m.ns) cursor_seek<GEN, HALF>(a, m, c);
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
// per-component select of two float4 (a ternary on the structs is lowered through a scratch copy)
__device__ __forceinline__ float4 sel4(bool c, const float4& x, const float4& y) {
    return make_float4(c ? x.x : y.x, c ? x.y : y.y, c ? x.z : y.z, c ? x.w : y.w);
}

struct StageRow {
    float u0[CPL], u1[CPL];   // u2^{k-1} of the row
    float z[CPL];             // z^k of the row
    float x2n[CPL];           // x2^k of the row
    int lk;                   // GEN: the row's lastk (its column segment's), set by the primal
};

template <bool EXACT, bool TRK, bool GEN = false, bool HALF = false>
__device__ __forceinline__ void stage_phase_a(const TvArgs& a, const float4& X2, const float4& U0,
                                              const float4& U1, const float4& YY, const float (&pu0)[CPL],
                                              StageRow& o, float& sd, float& sn, int nreal = CPL) {
    const float x2o[CPL] = {X2.x, X2.y, X2.z, X2.w};
    const float yy[CPL] = {YY.x, YY.y, YY.z, YY.w};
    o.u0[0] = U0.x; o.u0[1] = U0.y; o.u0[2] = U0.z; o.u0[3] = U0.w;
    o.u1[0] = U1.x; o.u1[1] = U1.y; o.u1[2] = U1.z; o.u1[3] = U1.w;
    // u1 of the column left of this lane's first column (lane-1's last); 0 at lane 0
    float u1l = __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(o.u1[CPL - 1]), 0x138 /* wave_shr:1 */, 0xF, 0xF, true));
    // HALF: lane 32 starts a window (the image's left edge or a halo cut: 0 either way)
    if (HALF && (threadIdx.x & 63) == 32) u1l = 0.f;
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
            // deepinv's constants as literal operands (psgla_common.hpp TV_*: fast kernels run only for them)
            xv = __builtin_fmaf(TV_TAU, yy[kk] - tt, xo) * TV_INV_OPT;
            zv = __builtin_fmaf(2.0f, xv, -xo);
            xn = __builtin_fmaf(TV_RHO, xv - xo, xo);
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
            const float v0 = __builtin_fmaf(TV_SIG, g0, uo0);
            const float v1 = __builtin_fmaf(TV_SIG, g1, uo1);
            const float s2 = __builtin_fmaf(v0, v0, v1 * v1);
            const float f = tv_proj_factor(vconst(a.ths), s2);
            un0[kk] = __builtin_fmaf(TV_RHO, __builtin_fmaf(v0, f, -uo0), uo0);
            un1[kk] = __builtin_fmaf(TV_RHO, __builtin_fmaf(v1, f, -uo1), uo1);
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
// FIRST (A1 only): stage 1, which reads its input row straight from the front's DMA staging (the row's front
// wave j % 4, slot (j / 4) % 3) instead of a ring -- a separate instantiation, so no stage branches on k around
// its LDS reads.
template <bool EXACT, bool TRK, bool GEN, bool A1, bool FIRST, bool HALF>
__device__ __forceinline__ void stage_loop(const TvArgs& a, StreamSharedT<A1>& sh, const RowMap& rm, int k, int n,
                                           int nsteps, int Qk, int lane, int lastk, int nreal, bool core, bool fresh) {
    // GEN: the lane's columns change with the column segment of the row (row split over virtual
    // planes): lastk / nreal / core follow the primal row's segment; each row carries its lastk
    // to its dual (StageRow.lk)
    auto set_geo = [&](int sgi) {
        if (GEN) {
            const SegGeo g = seg_geo<GEN, HALF>(a, rm.pl(sgi), lane >> 5);
            const int gj = g.f0 + CPL * lcol<HALF>(lane);
            lastk = a.W - 1 - gj;
            nreal = min(CPL, max(0, a.W - gj));
            core = g.on && gj < a.W && gj >= g.cc0 && gj < g.cc1;
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
            if (HALF) {                              // one sum per half-wave (each its own item / chain)
                const float2 rs = row_sum2(core ? lsd : 0.f, core ? lsn : 0.f);
                const int xi = __float_as_int(rs.x), yi = __float_as_int(rs.y);
                float d0 = __int_as_float(__builtin_amdgcn_readlane(xi, 0)) + __int_as_float(__builtin_amdgcn_readlane(xi, 16));
                float d1 = __int_as_float(__builtin_amdgcn_readlane(xi, 32)) + __int_as_float(__builtin_amdgcn_readlane(xi, 48));
                const float q0 = __int_as_float(__builtin_amdgcn_readlane(yi, 0)) + __int_as_float(__builtin_amdgcn_readlane(yi, 16));
                const float q1 = __int_as_float(__builtin_amdgcn_readlane(yi, 32)) + __int_as_float(__builtin_amdgcn_readlane(yi, 48));
                if (!EXACT) { d0 *= a.rho * a.rho; d1 *= a.rho * a.rho; }
                if (lane == 0) {
                    sh.red[sacc][0][k - 1][0] = d0; sh.red[sacc][0][k - 1][1] = q0;
                    sh.red[sacc][1][k - 1][0] = d1; sh.red[sacc][1][k - 1][1] = q1;
                }
            } else {
                float d = wave_sum(core ? lsd : 0.f);
                const float q = wave_sum(core ? lsn : 0.f);
                if (!EXACT) d *= a.rho * a.rho;          // fast sums hold (x - x2_prev)^2
                if (lane == 0) { sh.red[sacc][0][k - 1][0] = d; sh.red[sacc][0][k - 1][1] = q; }
            }
            lsd = 0.f; lsn = 0.f;
        }
    };
    auto primal = [&](int j, const float4& X2, const float4& U0, const float4& U1, const float4& YY,
                      const float (&pu0)[CPL], StageRow& cur) {
        float rd = 0.f, rn = 0.f;
        stage_phase_a<EXACT, TRK, GEN, HALF>(a, X2, U0, U1, YY, pu0, cur, rd, rn, nreal);
        if (GEN) cur.lk = lastk;
        if (TRK && j >= qc0 && j < qc1) { lsd += rd; lsn += rn; }
    };
    int t = 0;
    for (; t < tbeg; ++t) step_barrier();
    const int rin = StreamSharedT<A1>::rk(k - 1), rout = StreamSharedT<A1>::rk(k);
    auto load_row = [&](int j, float4& X2, float4& U0, float4& U1, float4& YY) {
        float4 A, B;
        YY = sh.y[j & (SP_YRING - 1)][lane];
        if (FIRST) {
            // the front's staging of row j (x2 = X, u2); a TV restart (fresh): x2 = Y, u2 = 0 (selects, no branch
            // around the LDS reads; lanes beyond the image read DMA'd values: they never feed an image column)
            const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 sX = sh.stX(j & 3, j)[lane];
            const float4 sA = sh.stUa(j & 3, j)[lane];
            const float4 sB = sh.stUb(j & 3, j)[lane];
            X2 = sel4(fresh, YY, sX);
            A = sel4(fresh, zero4, sA);
            B = sel4(fresh, zero4, sB);
        } else {
            const int sl = j & 1;
            X2 = sh.x2[rin][sl][lane];
            A = sh.ua[rin][sl][lane];
            B = sh.ub[rin][sl][lane];
        }
        U0 = make_float4(A.x, A.z, B.x, B.z);
        U1 = make_float4(A.y, A.w, B.y, B.w);
    };
    auto store_row = [&](int i, const StageRow& r, const float (&un0)[CPL], const float (&un1)[CPL]) {
        const int so = i & 1;
        sh.x2[rout][so][lane] = make_float4(r.x2n[0], r.x2n[1], r.x2n[2], r.x2n[3]);
        sh.ua[rout][so][lane] = make_float4(un0[0], un1[0], un0[1], un1[1]);
        sh.ub[rout][so][lane] = make_float4(un0[2], un1[2], un0[3], un1[3]);
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
// handling of such rows, compiled only into the kernels that need it
template <bool EXACT, bool ALPHA1, bool GEN, bool HALF>
__device__ __forceinline__ void stream_pass(const TvArgs& a, StreamSharedT<ALPHA1>& sh, const RowMap& rm, const int n,
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
    const int Q = rm.Q;
    const int qc0 = rm.htop, qc1 = Q - rm.hbot;          // core stream rows
    // column geometry of the first row's segment (the only one without GEN)
    const SegGeo g0 = seg_geo<GEN, HALF>(a, rm.pl0, lane >> 5);
    const int cc0 = g0.cc0, cc1 = g0.cc1;
    const int lc = lcol<HALF>(lane);
    const int gj0 = g0.f0 + CPL * lc;
    const bool lane_ok = g0.on && gj0 < W;
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
        int gjf = gj0;                                      // first column of the lane in row q (GEN:
        bool okf = lane_ok;                                 // per column segment)
        const float* xin = a.x[par_in];
        const float* u2in = a.u2[par_in];
        const float* x2in = ALPHA1 ? nullptr : a.x2[par_in];
        // The loads of a row are LDS-DMA'd 4 steps before the row is consumed (double-buffered
        // per front wave), row and column clamped into the plane so every lane loads.
        const int gjc = min(gj0, L - CPL);
        RowCursor rc_cur, rc_dma;
        cursor_init<GEN, HALF>(a, rm, rc_cur, min(fw, Q - 1));
        cursor_init<GEN, HALF>(a, rm, rc_dma, min(fw, Q - 1));
        // part `part` of the loads of stream row q: 0 = X, 1 = y, 2 = u2 (two halves), 3 = mask (+ x2)
        auto front_issue = [&](int part, int q, const RowCursor& rc) {
            const int rr = min(rc.r, H - 1);
            const int bi = (q >> 2) & 1;
            const int gjr = GEN ? min(rc.g.f0 + CPL * lc, L - CPL) : gjc;
            // 64-bit per-lane addresses (the SGPR-base form measured +12 % in round 2:
            // this kernel's row cursor sits in VGPRs, so each DMA pays two readfirstlane + 5 wait states)
            const size_t roff = (size_t)rr * L + gjr;
            const size_t base = rc.g.pbase + roff;
            if (part == 0) {
                glds16(xin + base, sh.stX(fw, q));
            } else if (part == 1) {
                glds16(a.yobs + rc.g.ybase + roff, sh.stY(fw, q));
            } else if (part == 2) {
                glds16(u2in + 2 * base, sh.stUa(fw, q));
                glds16(u2in + 2 * base + 4, sh.stUb(fw, q));
            } else {
                if (!ALPHA1) glds16(x2in + base, sh.stX2(fw, q));
                glds4(a.mask + rc.g.mbase + roff, &sh.fmk[fw][bi][0]);
            }
        };
        // row fw's loads up front; afterwards the loads of row q + 4 are issued one part per
        // phase of row q (into the buffer of row q - 4, consumed before phase 0 of row q), so
        // their issue cost is spread over four steps
        for (int part = 0; part < 4; ++part) front_issue(part, fw, rc_dma);
        cursor_advance<GEN, HALF>(a, rm, rc_dma, min(4, max(0, Q - 1 - fw)));
        // ======================= FRONT =======================
        // Row q (q % 4 == fw) runs its four phases in steps q .. q + 3: the loop below is unrolled by
        // phase (one step barrier after each), so no step decides its phase at run time.
        int t = 0;
        for (; t < fw && t < nsteps; ++t) step_barrier();
        for (int q = fw; q < Q; q += 4) {
            // ---- phase 0: Philox of row q; DMA part 0 of row q + 4
            front_issue(0, q + 4, rc_dma);
            {
                const RowGeo& g = rc_cur.g;
                if (GEN) {                                  // this row's segment's lanes
                    gjf = g.f0 + CPL * lc;
                    okf = g.on && gjf < W;
                }
                // psgla noise v2: the lane's 4 columns (gjf a multiple of 4) are one quad of the row, for
                // any W and independent of the row pitch
                uint32_t c0 = noise_quad(g.rbase + (size_t)rc_cur.r, gjf, W), c1 = (uint32_t)step,
                         c2 = TAG_LANGEVIN, c3 = (uint32_t)(a.seed >> 32);
                philox4x32_10(c0, c1, c2, c3, (uint32_t)a.seed, (uint32_t)(a.chain0 + g.bb));
                ph0 = c0; ph1 = c1; ph2 = c2; ph3 = c3;
            }
            step_barrier();
            // ---- phase 1: Box-Muller pair 1; DMA part 1
            front_issue(1, q + 4, rc_dma);
            box_muller(ph0, ph1, zn0, zn1);
            step_barrier();
            // ---- phase 2: Box-Muller pair 2; DMA part 2
            front_issue(2, q + 4, rc_dma);
            box_muller(ph2, ph3, zn2, zn3);
            step_barrier();
            // ---- phase 3: data term of row q -> ring 0 / Y ring; DMA part 3 of row q + 4
            {
                wait_vm<4>();   // row q's loads landed; parts 0-2 of row q + 4 may fly
                const int bi = (q >> 2) & 1;
                const float4 fX = sh.stX(fw, q)[lane];
                const float4 fYo = sh.stY(fw, q)[lane];
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
                if (!ALPHA1) {
                    // ring 0 = (x2, u2) of the staging; a TV restart (fresh): Y and 0 (reads first, then selects)
                    const float4 sX2 = sh.stX2(fw, q)[lane];
                    const float4 sA = sh.stUa(fw, q)[lane];
                    const float4 sB = sh.stUb(fw, q)[lane];
                    const float4 x2s = sel4(okf, sel4(fresh, Y4, sX2), zero4);
                    const int s0 = q & 1;
                    sh.x2[0][s0][lane] = x2s;
                    sh.ua[0][s0][lane] = sel4(fresh, zero4, sA);
                    sh.ub[0][s0][lane] = sel4(fresh, zero4, sB);
                }
                sh.y[q & (SP_YRING - 1)][lane] = Y4;
                // the wave's next rows: noise row q + 4, DMA of row q + 8... issued as q + 4
                front_issue(3, q + 4, rc_dma);
                cursor_advance<GEN, HALF>(a, rm, rc_cur, 4);
                if (q + 8 < Q) cursor_advance<GEN, HALF>(a, rm, rc_dma, 4);
            }
            step_barrier();
            t += 4;
        }
        for (; t < nsteps; ++t) step_barrier();
    } else if (role == 1) {
        // ---------------- STAGE (one inner TV iteration per wave) ----------------
        // the only column whose forward difference is forced to 0 is the image's right edge;
        // the left edge, the last row of u2[...,0] and the last column of u2[...,1] need no
        // select: the DPP shift feeds 0 at lane 0 and TV keeps those dual components exactly 0.
        const int lastk = W - 1 - gj0;                    // in 0..3 on the lane holding column W-1
        const int nreal = min(CPL, max(0, W - gj0));      // real (non-pitch-padding) columns of the lane
        __builtin_amdgcn_s_setprio(1);
        const int qk = stage_rows(k_st);
        if (ALPHA1 && k_st == 1) stage_loop<EXACT, false, GEN, ALPHA1, true, HALF>(a, sh, rm, k_st, n, nsteps, qk, lane, lastk, nreal, core, fresh);
        else if (trk) stage_loop<EXACT, true, GEN, ALPHA1, false, HALF>(a, sh, rm, k_st, n, nsteps, qk, lane, lastk, nreal, core, fresh);
        else stage_loop<EXACT, false, GEN, ALPHA1, false, HALF>(a, sh, rm, k_st, n, nsteps, qk, lane, lastk, nreal, core, fresh);
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
        cursor_init<GEN, HALF>(a, rm, rc_cur, min(bw, Q - 1));
        cursor_init<GEN, HALF>(a, rm, rc_dma, min(bw, Q - 1));
        auto back_issue = [&](int q, const RowCursor& rc) {
            if (need_prev) {
                const int rr = min(rc.r, H - 1);
                const int bi = (q >> 1) & 1;
                const int gjr = GEN ? min(rc.g.f0 + CPL * lc, L - CPL) : gjc;
                const size_t base = rc.g.pbase + (size_t)rr * L + gjr;
                glds16(mean_in + base, &sh.bst[bw][bi][0][0]);
                glds16(sq_in + base, &sh.bst[bw][bi][1][0]);
            }
        };
        // vector-memory stores per core row (all lanes of a wave store together; lane 0 is core)
        const int nst = 3 + (ALPHA1 ? 0 : 1) + ((si.acc && (si.blockend || si.liveout)) ? 2 : 0) + (si.sample ? 1 : 0);
        // a row's stores are spread over the wave's two steps: state + accumulators, then the rest
        bool hold = false, hcore = core;
        size_t h_base = 0;                  // per-lane element index
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
        if (bw + 2 < Q) cursor_advance<GEN, HALF>(a, rm, rc_dma, 2);
        back_issue(bw + 2, rc_dma);
        int c1 = 2, c2 = 0;
        // ======================= BACK =======================
        // Row q (q % 2 == bw) leaves the pipeline at step q + 4 + 3n (stage n wrote ring n row q in the step
        // before); its accumulator / sample stores go out in the wave's next step.  Unrolled by those two
        // steps (a step barrier after each), so no step decides at run time whether it has a row.
        int t = 0;
        const int t0 = 4 + 3 * n + bw;
        for (; t < t0 && t < nsteps; ++t) step_barrier();
        for (int q = bw; q < Qb && t < nsteps; q += 2) {
            {
                const int sl = q & 1;
                // stage n wrote ring n row q at step t - 1
                const int rn = StreamSharedT<ALPHA1>::rk(n);
                const float4 X2 = sh.x2[rn][sl][lane];
                const float4 UA = sh.ua[rn][sl][lane];
                const float4 UB = sh.ub[rn][sl][lane];
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
                cursor_advance<GEN, HALF>(a, rm, rc_cur, 2);
                if (q + 4 < Q) cursor_advance<GEN, HALF>(a, rm, rc_dma, 2);
                back_issue(q + 4, rc_dma);   // into the buffer just consumed (rows q, q + 4 share it)
                asm volatile("" ::: "memory");
                const bool rowcore = q >= qc0 && q < qc1;
                {
                    const int ns = rowcore ? nst : 0;   // this row's stores (both steps)
                    c1 = c2 + 2 + ns;
                    c2 = ns;
                }
                // GEN: the lanes' columns of this row's segment
                const int gjr = GEN ? rc.g.f0 + CPL * lc : gj0;
                const bool corer = GEN ? (rc.g.on && gjr < W && gjr >= rc.g.cc0 && gjr < rc.g.cc1) : core;
                if (rowcore && corer) {
                    const size_t base = rc.g.pbase + (size_t)rc.r * L + gjr;
                    st_nt(a.x[par_out] + base, Xo);
                    float* u2o = a.u2[par_out] + 2 * base;
                    st_nt(u2o, UA);
                    st_nt(u2o + 4, UB);
                    if (!ALPHA1) st_nt(a.x2[par_out] + base, X2);
                    // the accumulator / sample stores go out in the wave's next (idle) step
                    h_base = base; hM = M4; hQ = Q4; hX = Xo;
                }
                hold = rowcore;
                if (GEN) hcore = corer;
            }
            step_barrier();
            ++t;
            if (t < nsteps) {
                if (hold) {
                    flush_held();
                    hold = false;
                }
                step_barrier();
                ++t;
            }
        }
        for (; t < nsteps; ++t) step_barrier();
        if (hold) flush_held();
    }

    // rel_err partial sums of this stream -> global, per segment's chain (deepinv's
    // early-stop test, per chain); the tracking stages wrote sh.red[segment][k - 1]
}

// The previous step's pending early-stop redo (rare; a.redo[0], set by that step's finaliser): this workgroup
// redoes, segment by segment, every segment of its row range whose chain stopped (a.redo[4 + g] < n_tv inner
// iterations) -- each segment with its halo rows as the main pass cut them, so the workgroups' core rows cover
// every stopped row once (HALF: each item of a pair alone, in both half-waves, as the serial recompute).  The
// redone step's inputs are intact (ping-pong state).  (Folding the redo into the main pass's call site, in a loop,
// measured +14 % per step: the loop keeps the row map live across the pipeline.)
template <bool EXACT, bool ALPHA1, bool GEN, bool HALF>
__device__ __forceinline__ void stream_redo(const TvArgs& a, StreamSharedT<ALPHA1>& sh, long long pstep, bool pfresh) {
    RowMap rm;
    build_rowmap(a, blockIdx.x, rm);
    const int nitems = a.B * a.C * a.st_nsegs;
    for (int s = 0; s < rm.ns; ++s) {
        for (int hh = 0; hh < (HALF ? 2 : 1); ++hh) {
            const int item = HALF ? 2 * rm.pl(s) + hh : rm.pl(s);
            if (item >= nitems) continue;
            const int nstop = __builtin_amdgcn_readfirstlane(a.redo[4 + (item / a.st_nsegs) / a.C]);
            if (nstop >= a.n_tv) continue;
            RowMap r1;
            r1.ns = 1;
            r1.Q = rm.qs(s + 1) - rm.qs(s);
            r1.htop = s == 0 ? rm.htop : 0;
            r1.hbot = s == rm.ns - 1 ? rm.hbot : 0;
            r1.q1 = r1.q2 = r1.q3 = r1.Q;
            r1.pl0 = HALF ? a.st_nvp + item : item;
            r1.pl1 = r1.pl2 = r1.pl3 = 0;
            r1.lo0 = rm.lo(s);
            r1.lo1 = r1.lo2 = r1.lo3 = 0;
            __syncthreads();
            stream_pass<EXACT, ALPHA1, GEN, HALF>(a, sh, r1, nstop, false, pstep, pfresh);
        }
    }
}

template <bool EXACT, bool ALPHA1, bool GEN, bool HALF>
__global__ void __launch_bounds__(TV_THREADS) tv_stream_kernel(const TvArgs a) {
    __shared__ StreamSharedT<ALPHA1> sh;
    __shared__ int s_stop[MAXG];
    __shared__ int s_flag, s_item, s_next;
    const int C = a.C;
    const long long step = launch_step(a);
    const bool fresh = launch_fresh(a);
    // the previous step's pending early-stop redo (rare): all workgroups in parallel, then one grid barrier;
    // launch_mask 4 (redo_only): the redo alone
    if (a.par_redo && (a.fin_inline || a.redo_only)) {
        const int pend = __builtin_amdgcn_readfirstlane(a.redo[0]);
        if (pend & 1) {
            stream_redo<EXACT, ALPHA1, GEN, HALF>(a, sh, step - 1, (pend & 2) != 0);
            if (!a.redo_only) grid_sync(a.redo + 1, a.arrive + 3);
        }
        if (a.redo_only) return;
    }
    {
        RowMap rm;
        build_rowmap(a, blockIdx.x, rm);
        stream_pass<EXACT, ALPHA1, GEN, HALF>(a, sh, rm, a.n_tv, true, step, fresh);
        if (!a.fin_inline) return;        // main-pass-only launch (kernel timing): no side effects
        // rel_err partial sums of this stream -> global, per segment's chain (deepinv's
        // early-stop test, per chain); the tracking stages wrote sh.red[segment][k - 1]
        lds_barrier();
        for (int tt = threadIdx.x; tt < SP_MAXSEG * 2 * SP_MAXST; tt += blockDim.x) {
            const int sg = tt / (2 * SP_MAXST), hh = (tt / SP_MAXST) & 1, it = tt % SP_MAXST;   // it = k - 1
            if (sg < rm.ns && (HALF || hh == 0) && it >= 2 && it <= a.n_tv - 2) {
                // virtual plane -> item -> plane (HALF: the half-wave's item; a disabled half has none)
                const int vp = rm.pl(sg);
                int item = vp;
                if (HALF) {
                    item = 2 * vp + hh;
                    if (item >= a.B * C * a.st_nsegs) continue;
                }
                const int pl = item / a.st_nsegs;
                const int g = a.per_chain_norm ? pl / C : 0;
                atomicAdd(&a.norms[((size_t)g * a.n_tv + it) * 2], (double)sh.red[sg][hh][it][0]);
                atomicAdd(&a.norms[((size_t)g * a.n_tv + it) * 2 + 1], (double)sh.red[sg][hh][it][1]);
            }
        }
    }
    // ---- step finalisation by the last workgroup to arrive (no second launch) ----
    // Every wave's stores and atomics complete, then -- only when the finaliser may re-stream chains in this launch
    // (the serial early-stop recompute, par_redo = 0) -- one agent release per workgroup (writes the XCD's dirty L2
    // lines back), then the arrival count.  With the parallel redo nothing in this launch reads another
    // workgroup's plain stores (the rel-err sums are agent atomics, complete at wait_vm0; the redo runs in the next
    // launch, after the kernel boundary): round 6, -1.8 % at 64 chains, profiles/r06zh_stream_norelease_ab.txt.  The
    // last workgroup acquires before reading the rel-err sums or re-streaming a chain.
    wait_vm0();
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!a.par_redo) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
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
    if (a.par_redo) {
        // parallel redo (next launch, or launch_mask 4): publish the stop counts and the pending flag, reset the
        // grid-barrier count (every workgroup of this launch passed it before its main pass)
        for (int g = threadIdx.x; g < G; g += blockDim.x) a.redo[4 + g] = s_stop[g];
        if (threadIdx.x == 0) {
            a.redo[1] = 0;
            a.redo[0] = s_item ? (1 | (fresh ? 2 : 0)) : 0;
        }
        s_next = 1 << 30;                     // (uniform: every thread writes it) no serial recompute
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
        // the virtual plane (plane, column segment); HALF: the item alone, in both half-waves
        plane_rowmap(a.H, HALF ? a.st_nvp + item : item, rm);
        const int nstop = __builtin_amdgcn_readfirstlane(s_stop[plane / C]);
        stream_pass<EXACT, ALPHA1, GEN, HALF>(a, sh, rm, nstop, false, step, fresh);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < a.B * a.n_tv * 2; i += blockDim.x) a.norms[i] = 0.0;
    if (threadIdx.x == 0) {
        *a.arrive = 0;
        if (a.fresh_dev) *a.fresh_dev = 0;
        if (a.advance_step && a.d_step) *a.d_step = *a.d_step + 1;   // (re-read: the start-of-kernel value measured +0.5 % here)
    }
}

int stream_blocks_per_cu(bool exact, bool alpha1, bool gen, bool half) {
    static int cache[16] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
    const int slot = (exact ? 8 : 0) | (alpha1 ? 4 : 0) | (gen ? 2 : 0) | (half ? 1 : 0);
#define PSGLA_STREAM_OCC(E, A, G, HF) \
    if (exact == E && alpha1 == A && gen == G && half == HF) \
        return occupancy_cached(cache, slot, reinterpret_cast<const void*>(&tv_stream_kernel<E, A, G, HF>), TV_THREADS);
    PSGLA_STREAM_OCC(true, true, false, false) PSGLA_STREAM_OCC(true, true, true, false) PSGLA_STREAM_OCC(true, false, false, false) PSGLA_STREAM_OCC(true, false, true, false)
    PSGLA_STREAM_OCC(false, true, false, false) PSGLA_STREAM_OCC(false, true, true, false) PSGLA_STREAM_OCC(false, false, false, false) PSGLA_STREAM_OCC(false, false, true, false)
    PSGLA_STREAM_OCC(true, true, true, true) PSGLA_STREAM_OCC(true, false, true, true) PSGLA_STREAM_OCC(false, true, true, true) PSGLA_STREAM_OCC(false, false, true, true)
#undef PSGLA_STREAM_OCC
    return 0;
}

void launch_stream(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen, bool half) {
#define PSGLA_STREAM(E, A, G, HF) \
    if (exact == E && alpha1 == A && gen == G && half == HF) { hipLaunchKernelGGL((tv_stream_kernel<E, A, G, HF>), grid, dim3(TV_THREADS), 0, st, s); return; }
    PSGLA_STREAM(true, true, false, false) PSGLA_STREAM(true, true, true, false) PSGLA_STREAM(true, false, false, false) PSGLA_STREAM(true, false, true, false)
    PSGLA_STREAM(false, true, false, false) PSGLA_STREAM(false, true, true, false) PSGLA_STREAM(false, false, false, false) PSGLA_STREAM(false, false, true, false)
    PSGLA_STREAM(true, true, true, true) PSGLA_STREAM(true, false, true, true) PSGLA_STREAM(false, true, true, true) PSGLA_STREAM(false, false, true, true)
#undef PSGLA_STREAM
}

}  // namespace psgla
