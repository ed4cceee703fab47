// Small-batch tile PSGLA + TV step (tv_tile_kernel): the strong-scaling split's per-GPU kernel and the
// reference's real image shapes at the CLI's batch sizes.
// (library overview: psgla_common.hpp)
#include "psgla_common.hpp"

namespace psgla {

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

template <int R, int NW>
struct TileShared {
    float4 zrow[NW][WAVE];             // first-row z of each wave (read by the wave above)
    float4 urow[NW][WAVE];             // last-row u2[..., 0] of each wave (read by the wave below)
    float4 mst[tile_mst_rows(NW, R)][2][WAVE];   // mean / sq of the tile's core rows (LDS-DMA after the data term)
    float2 red[MAXIT][NW][4];          // rel_err partial sums per (iteration, wave, 16-lane row of the wave)
    int s_stop[MAXG];
    int s_flag, s_item, s_next;
    int s_uncert;                      // this tile's rel-err partials do not rule out a stop (below)
    int s_nuncert;                     // finaliser: tiles whose partials do not rule out a stop
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
    const int cc1 = GEN ? (seg == a.st_nsegs - 1 ? W : min(W, cc0 + a.st_seg_w)) : W;   // the last segment: the rest
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
    // ---- 1. every load the first iteration needs in flight: state, observation and mask to registers
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
    // ---- 2. the noise of the tile's rows (no memory dependence: overlaps the loads)
    float Zn[R][CPL];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        // psgla noise v2: the lane's 4 columns (from a multiple of 4) are one quad of the row, for any W and
        // independent of the row pitch
        normal_quad(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step, TAG_LANGEVIN,
                    noise_quad((size_t)c * H + (rv[r] ? gi[r] : 0), gj0, W), Zn[r]);
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
    // The previous mean / sq of the core rows, LDS-DMA'd only now (round 4): the accumulator update after the last
    // iteration is their only reader, so these 8 B per element land during the iterations instead of competing
    // with the loads above, which the first iteration waits for.  The iteration barriers drain LDS only
    // (lgkmcnt), so nothing waits for this DMA before store_x_side's vmcnt(0).
    if (need_prev && n_it >= 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (rv[r] && core[r]) {
                const size_t base = poff + (size_t)gi[r] * L + gjc;
                const int ro = (gi[r] - r0) * (int)sizeof(sh.mst[0]);
                glds16_at(a.mean[par_in] + base, &sh.mst[0][0][0], ro);
                glds16_at(a.sq[par_in] + base, &sh.mst[0][1][0], ro);
            }
        }
    }

    // ---- 4. inner TV iterations (deepinv 0.2.1 TVDenoiser, the stream kernel's arithmetic)
    const bool lastlane = gj0 + CPL == W;              // holds column W-1: no forward difference there
    // fast mode (round 5): the horizontal difference's sigma per lane column, 0 at column W-1 -- a per-lane constant
    // instead of a select per element and iteration (the same value: sigma * finite == 0 there)
    float sg1[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) sg1[k] = (GEN ? lastk == k : (k == CPL - 1 && lastlane)) ? 0.f : TV_SIG;
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
    // TM: whether the iteration's rel-err terms are tracked -- 0 no, 1 yes (compile time: the loops below run the
    // untracked and tracked iterations as separate straight-line bodies), 2 decided at run time (the peeled last one)
    auto iteration = [&](const int it, auto last_tag, auto tm_tag) {
        constexpr bool LAST = decltype(last_tag)::value;
        constexpr int TM = decltype(tm_tag)::value;
        const bool trk = TM == 2 ? (track && it >= trk_lo(a) && it <= trk_hi(a)) : TM == 1;
        float sd = 0.f, sn = 0.f;
        const int span = n_it - 1 - it;
        const bool act_p = wr1 > r0 - span && wr0 < r1 + span + 1;
        const bool act_d = wr1 > r0 - span && wr0 < r1 + span;
        // primal: x = prox_tau_fx(x2 - tau nabla^T u2, Y); z = 2x - x2; x2 += rho (x - x2)
        const float4 up = (w > 0) ? sh.urow[w - 1][lane] : zero4;
        // the wave's first row -- the only one reading the hand-off from the wave above -- last, so that LDS
        // read's latency hides behind the other rows (-0.9 % at 8 chains, profiles/r03o_tile_row0_last_ab.txt)
        if (act_p) {
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
            const int r = (rr + 1) % R;
            const float u1l = __int_as_float(
                __builtin_amdgcn_update_dpp(0, __float_as_int(u1[r][CPL - 1]), 0x138 /* wave_shr:1 */, 0xF, 0xF, true));
            float rd = 0.f, rn = 0.f;                      // fast: the row's rel-err terms (as the row stream)
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
                    // deepinv's constants as literal operands (psgla_common.hpp TV_*; round 6)
                    xv = __builtin_fmaf(TV_TAU, yv[r][k] - tt, xo) * TV_INV_OPT;
                    zv = __builtin_fmaf(2.0f, xv, -xo);
                    xn = __builtin_fmaf(TV_RHO, xv - xo, xo);
                }
                // rel-err terms of the counted rows (row-uniform test; lanes past W are masked once, at
                // the reduction: adding nothing and adding +0 leave a lane's sum identical).  Fast mode (round 5):
                // every row's terms into its own partial sums, added once per row -- a per-element select of the
                // running sums cost 2 VALU per element (the row stream's order)
                const bool real = !GEN || k < nreal;       // padding columns are not part of the norms
                if (EXACT) {
                    if (trk && core[r] && rv[r]) {
                        const float d = real ? xo - xn : 0.f;
                        const float q = real ? xn + 1e-12f : 0.f;
                        sd = __builtin_fmaf(d, d, sd);
                        sn = __builtin_fmaf(q, q, sn);
                    }
                } else if (trk) {
                    const float d = real ? xv - xo : 0.f;
                    const float q = real ? xn : 0.f;
                    rd = __builtin_fmaf(d, d, rd);
                    rn = __builtin_fmaf(q, q, rn);
                }
                z[r][k] = zv;
                x2[r][k] = xn;
            }
            if (!EXACT && trk && core[r] && rv[r]) {
                sd += rd;
                sn += rn;
            }
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
        if (act_d) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float zr3 = __int_as_float(
                __builtin_amdgcn_update_dpp(0, __float_as_int(z[r][0]), 0x130 /* wave_shl:1 */, 0xF, 0xF, true));
            const bool down = gi[r] < H - 1;
            // fast mode (round 5): the plane's last row (no vertical difference) takes sigma 0 in its dual -- a
            // row-uniform scalar instead of a per-element select (the same value: sigma * 0 == 0 * finite)
            // (a.sig_tv == TV_SIG in the fast mode; a select between the literal and 0 made the register allocator
            // spill a VGPR in the 48-row instance, round 6)
            const float sg0 = down ? a.sig_tv : 0.f;
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
                    const float v0 = __builtin_fmaf(sg0, zd - zc, uo0);
                    const float v1 = __builtin_fmaf(sg1[k], zr - zc, uo1);
                    const float s2 = __builtin_fmaf(v0, v0, v1 * v1);
                    const float f = tv_proj_factor(vconst(a.ths), s2);
                    u0[r][k] = __builtin_fmaf(TV_RHO, __builtin_fmaf(v0, f, -uo0), uo0);
                    u1[r][k] = __builtin_fmaf(TV_RHO, __builtin_fmaf(v1, f, -uo1), uo1);
                }
            }
        }
        }
        if (act_d) sh.urow[w][lane] = make_float4(u0[R - 1][0], u0[R - 1][1], u0[R - 1][2], u0[R - 1][3]);
        __syncthreads();
    };
    // iterations [0, t0) and [t1, n_it - 1) untracked, [t0, t1) tracked (round 5: one loop with a run-time test
    // merged both paths and paid register copies for it on every iteration), the last one peeled
    {
        using TM0 = std::integral_constant<int, 0>;
        using TM1 = std::integral_constant<int, 1>;
        const int nl = max(n_it - 1, 0);
        const int t0 = track ? min(max(trk_lo(a), 0), nl) : nl;
        const int t1 = track ? min(max(trk_hi(a) + 1, t0), nl) : nl;
        for (int it = 0; it < t0; ++it) iteration(it, std::false_type{}, TM0{});
        for (int it = t0; it < t1; ++it) iteration(it, std::false_type{}, TM1{});
        for (int it = t1; it < nl; ++it) iteration(it, std::false_type{}, TM0{});
    }
    if (n_it > 0) iteration(n_it - 1, std::true_type{}, std::integral_constant<int, 2>{});
    // ---- 5. rel_err partial sums -> the chain's norms (one fp64 atomic per iteration and workgroup)
    if (track) {
        // (on wave 0, before the u2 stores: spreading the sums over waves delays every wave's u2 stores -- 8
        // chains +4.3 %, castle at batch 1 +9 % -- and moving them after the u2 stores gains nothing:
        // profiles/r04l_tile_ab.txt, r04m_tile_ab.txt)
        const int t = threadIdx.x;
        if (t >= trk_lo(a) && t <= trk_hi(a) && t < n_it) {
            double sd = 0.0, sn = 0.0;
            for (int ww = 0; ww < NW; ++ww)
                for (int q = 0; q < 4; ++q) { sd += sh.red[t][ww][q].x; sn += sh.red[t][ww][q].y; }
            if (!EXACT) sd *= (double)(a.rho * a.rho);     // fast sums hold (x - x2_prev)^2
            // Round 6: deepinv stops when ||x2 - x2_prev|| < tol ||x2||, i.e. sum(d) < tol^2 sum(n) over the chain's
            // tiles.  A tile whose own partials satisfy d >= tol^2 (1 + 1e-5) n cannot contribute to a stop; when no
            // tile of the launch reports otherwise (the arrival count's high half), the finaliser knows that no chain
            // stopped without reading the sums (the 1e-5 margin covers the fp64 sums and the fp32 sqrt / divide of
            // the test, whose rounding is below 1e-6 relative)
            if (!(sd >= ((double)a.tol * (double)a.tol) * (1.0 + 1e-5) * sn)) sh.s_uncert = 1;
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
    // u2 out.  A lane's 4 columns are 32 contiguous bytes of u2 (deepinv's (.., W, 2) layout): halves A (columns
    // 0-1) and B (2-3).  Stored as they lie, each dwordx4 instruction would write every other 16 B of a 2 KB span
    // -- with write-through (sc1) stores that is partial-line traffic (PMC: 1.39x the algorithmic write bytes,
    // VERDICT r3).  Instead B moves to the other half-wave (v_permlane32_swap): the first instruction writes
    // lanes 0-31's A and B (one contiguous 1 KB), the second lanes 32-63's.
    {
        const bool lo = lane < 32;
        const int gjo = f0 + CPL * (lane ^ 32);                 // columns of the lane whose B this lane stores
        const bool corelane_o = GEN ? (gjo < W && gjo >= cc0 && gjo < cc1) : gjo < W;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!(rv[r] && core[r])) continue;
            const size_t row = poff + (size_t)gi[r] * L;
            float* const u2r = a.u2[par_out] + 2 * row;
            const float4 A = make_float4(u0[r][0], u1[r][0], u0[r][1], u1[r][1]);
            const float Bv[4] = {u0[r][2], u1[r][2], u0[r][3], u1[r][3]};
            float Bs[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_int(Bv[k]), __float_as_int(Bv[k]), false, false);
                Bs[k] = __int_as_float(lo ? sw[1] : sw[0]);   // lanes 0-31: B of lane + 32; lanes 32-63: of lane - 32
            }
            const float4 B4 = make_float4(Bs[0], Bs[1], Bs[2], Bs[3]);
            float* const pa = u2r + 2 * gj0;                     // own A
            float* const pb = u2r + 2 * gjo + 4;                 // the other lane's B
            // (per-component selects: a ternary on the float4 structs is lowered through a scratch copy)
            const float4 v1 = make_float4(lo ? A.x : B4.x, lo ? A.y : B4.y, lo ? A.z : B4.z, lo ? A.w : B4.w);
            const float4 v2 = make_float4(lo ? B4.x : A.x, lo ? B4.y : A.y, lo ? B4.z : A.z, lo ? B4.w : A.w);
            if (lo ? corelane : corelane_o) st_tile(lo ? pa : pb, v1);
            if (lo ? corelane_o : corelane) st_tile(lo ? pb : pa, v2);
        }
    }
}

template <bool EXACT, bool ALPHA1, int R, bool GEN, int NW>
__global__ void __launch_bounds__(NW * WAVE) tv_tile_kernel(const TvArgs a) {
    __shared__ TileShared<R, NW> sh;
    constexpr bool SPLIT = NW == 8;                    // two-phase arrival (below)
    const long long step = launch_step(a);
    const bool fresh = launch_fresh(a);
    if (threadIdx.x == 0) sh.s_uncert = 0;             // (read after sb_tile's barriers)
    const int P = a.B * a.C;
    const int T = a.nbands * (GEN ? a.st_nsegs : 1);  // tiles per plane: (column segment, band)
    {
        // the P * T tiles, plane-major, cut into 8 runs, one per XCD (blocks x and x + 8 share one):
        // the tiles of a plane share an XCD's L2 for their halo rows, and every XCD gets work even when
        // there are fewer than 8 planes (one image at the CLI's batch 1)
        // (round 5: runs of floor(N / 8) or ceil(N / 8) tiles -- the first N % 8 runs one longer -- on a grid of
        // exactly N workgroups: no workgroup without a tile)
        const int N = P * T, q8 = N >> 3, r8 = N & 7;
        const int x = blockIdx.x, xcd = x & 7, k = x >> 3;
        const int item = xcd * q8 + min(xcd, r8) + k;
        // The previous step's pending early-stop redo (rare; a.redo[0], published by that step's finaliser; round 5):
        // every workgroup whose chain stopped redoes its own tile of that step with the stopped iteration count
        // (the step's inputs are intact: ping-pong state), all in parallel, then one grid barrier before this
        // step reads them.  launch_mask 4 (redo_only): the redo alone.
        if (a.par_redo && (a.fin_inline || a.redo_only)) {
            const int pend = __builtin_amdgcn_readfirstlane(a.redo[0]);
            if (pend & 1) {
                if (item < N) {
                    const int plane = item / T, t = item - plane * T;
                    const int seg = GEN ? t / a.nbands : 0;
                    const int band = t - seg * a.nbands;
                    const int nstop = __builtin_amdgcn_readfirstlane(a.redo[4 + plane / a.C]);
                    if (nstop < a.n_tv)
                        sb_tile<EXACT, ALPHA1, R, GEN, NW>(a, sh, plane, seg, band, nstop, false, step - 1,
                                                           (pend & 2) != 0, [] {});
                }
                if (!a.redo_only) grid_sync(a.redo + 1, a.arrive + 3);
            }
            if (a.redo_only) return;
        }
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
                // (one-phase arrival: the high half counts the tiles whose rel-err partials leave a stop possible)
                const int unc = SPLIT ? 0 : (sh.s_uncert ? 1 : 0);
                const int old = __hip_atomic_fetch_add(a.arrive, 1 + (unc << 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                sh.s_flag = ((old & 0xFFFF) == (int)gridDim.x - 1) ? 1 : 0;
                sh.s_nuncert = SPLIT ? 1 : (old >> 16) + unc;
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
    const int ncp = a.norm_copies;
    // Round 6: no tile left a stop possible (its rel-err partials, above: the arrival count's high half) -- the common
    // case -- so no chain stopped: the sums are only zeroed for the next step and the pending word cleared, by
    // stores with no barrier after them (a __syncthreads waits for the stores before it: ~1 us)
    if (sh.s_nuncert == 0) {
        const size_t cstride = (size_t)a.B * a.n_tv * 2;
        for (int i = threadIdx.x; i < G * MAXIT * ncp; i += blockDim.x) {
            const int gt = i / ncp, cp = i - gt * ncp;
            const int g = gt / MAXIT, t = gt - g * MAXIT;
            if (t >= trk_lo(a) && t <= trk_hi(a) && t < a.n_tv) {
                double* const n0 = a.norms + (size_t)cp * cstride + ((size_t)g * a.n_tv + t) * 2;
                __hip_atomic_store(n0, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(n0 + 1, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (a.par_redo && threadIdx.x == 0) {
            a.redo[1] = 0;
            a.redo[0] = 0;
        }
        // the stores complete before the resets below (measured: without this wait 8 chains +0.7 %, castle at batch 1
        // -2.6 %; with it 0 % / -3.8 % against the full finalisation, profiles/r06ze_tile_nostop_ab.txt)
        wait_vm0();
    } else {
    for (int g = threadIdx.x; g < G; g += blockDim.x) sh.s_stop[g] = 0;
    // Few chains with several norm copies (the CLI's castle at batch 1-4: 8 copies): every (chain, iteration, copy)
    // pair is read by its own thread -- two exchanges per lane, issued by a few wave-instructions -- into LDS
    // (sh.red is free here), then summed in copy order by one thread per (chain, iteration): the same sums as the
    // per-(chain, iteration) loop below, whose 16 exchanges per lane issue one after another (round 6)
    constexpr int RED_D = (int)(sizeof(sh.red) / sizeof(double));
    const bool spread = ncp > 1 && ncp <= 8 && G * MAXIT * ncp * 2 <= RED_D;
    double* const cpv = reinterpret_cast<double*>(&sh.red[0][0][0]);
    if (spread) {
        const size_t cstride = (size_t)a.B * a.n_tv * 2;
        for (int i = threadIdx.x; i < G * MAXIT * ncp; i += blockDim.x) {
            const int gt = i / ncp, cp = i - gt * ncp;
            const int g = gt / MAXIT, t = gt - g * MAXIT;
            if (t >= trk_lo(a) && t <= trk_hi(a) && t < a.n_tv) {
                double* const n0 = a.norms + (size_t)cp * cstride + ((size_t)g * a.n_tv + t) * 2;
                cpv[2 * i] = __hip_atomic_exchange(n0, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                cpv[2 * i + 1] = __hip_atomic_exchange(n0 + 1, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < G * MAXIT; i += blockDim.x) {
        const int g = i / MAXIT, t = i - g * MAXIT;
        if (spread && t >= trk_lo(a) && t <= trk_hi(a) && t < a.n_tv) {
            double nd = 0.0, nn = 0.0;
            for (int cp = 0; cp < ncp; ++cp) { nd += cpv[2 * (i * ncp + cp)]; nn += cpv[2 * (i * ncp + cp) + 1]; }
            const float rel = (float)sqrt(nd) / (float)sqrt(nn);
            if (rel < a.tol) atomicOr(&sh.s_stop[g], 1 << t);
        } else if (!spread && t >= trk_lo(a) && t <= trk_hi(a) && t < a.n_tv) {
            // read by agent-scope atomics (exchange with 0.0: read and reset in one operation), as they were
            // written: 8-B agent atomics on both sides of the hand-off, performed where the producers' adds were
            // With several copies, the first 8 copies' reads are issued back to back and waited for once (round 4:
            // one round trip instead of one per copy: castle at batch 1 -4.8 %, profiles/r04k_tile_fin_ab.txt),
            // then added in copy order as before; one copy keeps the plain pair of reads
            const size_t cstride = (size_t)a.B * a.n_tv * 2;
            double* const n0 = a.norms + ((size_t)g * a.n_tv + t) * 2;
            double nd = 0.0, nn = 0.0;
            if (a.norm_copies == 1) {
                nd += __hip_atomic_exchange(n0, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                nn += __hip_atomic_exchange(n0 + 1, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                double vd[8], vn[8];
#pragma unroll
                for (int cp = 0; cp < 8; ++cp) {
                    vd[cp] = vn[cp] = 0.0;
                    if (cp < a.norm_copies) {
                        vd[cp] = __hip_atomic_exchange(n0 + cp * cstride, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        vn[cp] = __hip_atomic_exchange(n0 + cp * cstride + 1, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
#pragma unroll
                for (int cp = 0; cp < 8; ++cp) {
                    if (cp < a.norm_copies) { nd += vd[cp]; nn += vn[cp]; }
                }
                for (int cp = 8; cp < a.norm_copies; ++cp) {   // beyond 8 copies (not used by the engine): in order
                    nd += __hip_atomic_exchange(n0 + cp * cstride, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    nn += __hip_atomic_exchange(n0 + cp * cstride + 1, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
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
    if (a.par_redo) {
        // parallel redo (next launch, or launch_mask 4): publish the stop counts and the pending flag, reset the
        // grid-barrier count (every workgroup of this launch passed it before its tile)
        for (int g = threadIdx.x; g < G; g += blockDim.x) a.redo[4 + g] = sh.s_stop[g];
        if (threadIdx.x == 0) {
            a.redo[1] = 0;
            a.redo[0] = sh.s_item ? (1 | (fresh ? 2 : 0)) : 0;
        }
    } else if (sh.s_item) {
        // rare: redo every tile of a stopped chain with the stopped iteration count (inputs intact), once every
        // other workgroup's stores are complete (phase 2; all of them have arrived, so each will count: bounded
        // wait only as a guard)
        if (SPLIT && threadIdx.x == 0) {
            bool done = false;
            for (int spin = 0; spin < (1 << 24) && !done; ++spin) {
                done = (__hip_atomic_load(a.arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 16) >= (int)gridDim.x - 1;
                if (!done) __builtin_amdgcn_s_sleep(2);
            }
            // the guard expired: the redo may race late first-pass stores -- record it for the host
            // (arrive[3], read by FusedTvChains.check_handoff()) instead of going on silently
            if (!done) __hip_atomic_store(a.arrive + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
    }
    // (the norm copies were zeroed by the exchanges that read them, or by the stores above; entries outside the
    // tracked iterations are never written)
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

int tile_blocks_per_cu(const TvArgs& s, bool exact, bool alpha1, bool gen) {
    static int cache[16] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
    const int slot = (exact ? 8 : 0) | (alpha1 ? 4 : 0) | (gen ? 2 : 0) | (s.tile_r == 3 ? 1 : 0);
#define PSGLA_TILE_OCC(E, A, NWV, RV) \
    if (exact == E && alpha1 == A && s.tile_nw == NWV && s.tile_r == RV) \
        return occupancy_cached(cache, slot, gen ? reinterpret_cast<const void*>(&tv_tile_kernel<E, A, RV, true, NWV>) \
                                                 : reinterpret_cast<const void*>(&tv_tile_kernel<E, A, RV, false, NWV>), NWV * WAVE);
    PSGLA_TILE_OCC(true, true, 16, 2) PSGLA_TILE_OCC(true, false, 16, 2) PSGLA_TILE_OCC(false, true, 16, 2) PSGLA_TILE_OCC(false, false, 16, 2)
    PSGLA_TILE_OCC(true, true, 16, 3) PSGLA_TILE_OCC(false, true, 16, 3)
#undef PSGLA_TILE_OCC
    return 0;
}

bool launch_tile(const TvArgs& s, dim3 grid, hipStream_t st, bool exact, bool alpha1, bool gen) {
#define PSGLA_TILE(E, A, NWV, RV) \
    if (exact == E && alpha1 == A && s.tile_nw == NWV && s.tile_r == RV) { \
        if (!gen) hipLaunchKernelGGL((tv_tile_kernel<E, A, RV, false, NWV>), grid, dim3(NWV * WAVE), 0, st, s); \
        else hipLaunchKernelGGL((tv_tile_kernel<E, A, RV, true, NWV>), grid, dim3(NWV * WAVE), 0, st, s);      \
        return true; \
    }
    // the instances select_step_kernel (api.hip) dispatches -- none spills a VGPR (round 6; checked by
    // tests/test_native_abi.py): 32-row tiles everywhere, 48-row tiles at alpha = 1 (alpha != 1 spilled 1-12 VGPRs);
    // no 72-row tiles (8 waves x 9 rows spilled 11-68 VGPRs at 256)
#define PSGLA_TILES(E, A) PSGLA_TILE(E, A, 16, 2)
    PSGLA_TILES(true, true) PSGLA_TILES(true, false) PSGLA_TILES(false, true) PSGLA_TILES(false, false)
    PSGLA_TILE(true, true, 16, 3) PSGLA_TILE(false, true, 16, 3)
#undef PSGLA_TILES
#undef PSGLA_TILE
    return false;
}

}  // namespace psgla
