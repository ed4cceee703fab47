// C ABI of the fused TV step (psgla_tv_step, psgla_tv_step_kernel, psgla_tv_prox): kernel selection, work
// split and launch; the error state shared by every entry point of the library.
// (library overview: psgla_common.hpp)
#include "psgla_common.hpp"

// =======================================================================================
// C ABI
// =======================================================================================
using namespace psgla;

thread_local char g_err[512] = "";

int fail(int code, const char* msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
    return code ? code : (int)hipErrorInvalidValue;
}

int launch_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return 0;
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

// The parallel early-stop redo meets at a grid barrier (grid_sync), so every workgroup of the grid must be resident at
// once: a grid within the CUs and within the instance's occupancy x the CUs.  Otherwise the finalising
// workgroup recomputes stopped chains serially.  (The barrier's spin is bounded: an expired guard sets arrive[3],
// which FusedTvChains.check_handoff raises on -- another process's kernels holding CUs for the whole guard is the
// case the occupancy query cannot see.)
static bool grid_resident(long long grid, int per_cu) {
    const long long cus = device_cus();
    return per_cu > 0 && grid <= cus && grid <= (long long)per_cu * cus;
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
// stay within the LDS staging of mean / sq (tile_mst_rows).  Returns the number of workgroups (one per tile),
// 0 if the shape does not fit (halo too large, no segmentation).
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
    return P * nb * nsegs;
}

// Column segments of the streaming kernel: core widths seg_w (a multiple of 4; the last segment takes the rest)
// cut from the image width W; segment s's window of `win` columns starts at f0 = (cc0 - h) & ~3 (cc0 = s * seg_w)
// and must reach cc1 + h for interior cuts (the TV dependency cone) and the row pitch L at the image's right end
// (no halo needed at the image edges).  Fewest segments (then the widest seg_w from ceil(W / n) down); 0 if none
// fits.  win = 256: a wave's window (4 columns x 64 lanes); 128: a half-wave's (st_half).
static int stream_segments(int W, int L, int h, int* seg_w, int win = TV_COLS) {
    for (int n = 1; n <= 64; ++n) {
        const int sw0 = (((W + n - 1) / n) + 3) & ~3;
        for (int sw = sw0; sw >= 4 && sw >= sw0 - 32; sw -= 4) {
            if ((long long)sw * (n - 1) >= W) continue;         // last segment would be empty
            bool ok = true;
            for (int sgi = 0; sgi < n && ok; ++sgi) {
                const int cc0 = sgi * sw, cc1 = (sgi == n - 1) ? W : min(W, cc0 + sw);
                const int f0 = max(0, cc0 - h) & ~3;
                const int need = (cc1 >= W) ? L : min(L, cc1 + h);
                ok = need - f0 <= win;
            }
            if (ok) {
                if (seg_w) *seg_w = sw;
                return n;
            }
        }
    }
    return 0;
}

template <bool EXACT, int FRONT, bool ALPHA1>
static int launch_tv(const TvArgs& a, hipStream_t st, int mask = 3) {
    const int P = a.B * a.C;
    if (mask == 0) mask = 3;
    // launch_mask 4: settle a pending early-stop redo of the last step (the kernel redoes the stopped chains' part
    // of it, nothing else), then clear the pending flag; only the stream / tile kernels with a redo buffer have one
    if (mask == 4) {
        if (FRONT != FRONT_INPAINT || !a.redo || (a.tile_r == 0 && !a.stream)) return 0;
        TvArgs s = a;
        s.fin_inline = 0;
        s.redo_only = 1;
        int rc;
        if (a.tile_r > 0) {
            const int grid = P * s.nbands * s.st_nsegs;
            const bool gen = !(s.ldw == s.W && s.st_nsegs == 1);
            s.par_redo = grid_resident(grid, tile_blocks_per_cu(s, EXACT, ALPHA1, gen)) ? 1 : 0;
            if (!s.par_redo) return 0;   // (the tile kernel's finaliser recomputed stopped chains itself)
            if (!launch_tile(s, dim3(grid), st, EXACT, ALPHA1, gen))
                return fail(0, "psgla_tv_step: internal error: no tile kernel of this shape");
            rc = launch_check("tv_tile_kernel(redo)");
        } else {
            const int grid = s.split_wgs > 0 ? s.split_wgs : s.st_nvp;
            s.par_redo = grid_resident(grid, stream_blocks_per_cu(EXACT, ALPHA1, !(s.ldw == s.W && s.st_nsegs == 1),
                                                                  s.st_half != 0)) ? 1 : 0;
            if (!s.par_redo) return 0;
            launch_stream(s, dim3(grid), st, EXACT, ALPHA1, !(s.ldw == s.W && s.st_nsegs == 1), s.st_half != 0);
            rc = launch_check("tv_stream_kernel(redo)");
        }
        if (rc) return rc;
        if (hipMemsetAsync(a.redo, 0, sizeof(int), st) != hipSuccess) return launch_check("psgla_tv_step(redo clear)");
        return 0;
    }
    if (mask & 1) {
        if (FRONT == FRONT_INPAINT && a.tile_r > 0) {
            TvArgs s = a;
            s.fin_inline = (mask & 2) ? 1 : 0;
            const int grid = P * s.nbands * s.st_nsegs;                   // tile_kernel: one workgroup per tile
            // (the two-phase arrival counter keeps a count of workgroups in 15 bits)
            if (grid > 32767) return fail(0, "psgla_tv_step: more than 32767 tiles in one launch");
            // several copies of the rel-err sums only where many tiles share a chain: with the finaliser's copy
            // reads issued back to back (round 4), 8 copies cost 8 chains of 30 tiles +1.6 % and save castle at
            // batch 2 (108 tiles per chain) 3.5 % and at batch 1 (246) 5 % (profiles/r04k_tile_fin_ab.txt)
            if (s.norm_copies < 1 || s.C * s.nbands * s.st_nsegs < 64) s.norm_copies = 1;
            // parallel early-stop redo when every tile is resident at once (its grid barrier); otherwise the
            // finalising workgroup recomputes stopped chains itself
            const bool gen = !(s.ldw == s.W && s.st_nsegs == 1);
            s.par_redo = (s.redo && grid_resident(grid, tile_blocks_per_cu(s, EXACT, ALPHA1, gen))) ? 1 : 0;
            if (launch_tile(s, dim3(grid), st, EXACT, ALPHA1, gen)) return launch_check("tv_tile_kernel");
            return fail(0, "psgla_tv_step: internal error: no tile kernel of this shape");
        }
        if (FRONT == FRONT_INPAINT && a.stream) {
            TvArgs s = a;
            s.fin_inline = (mask & 2) ? 1 : 0;
            const int grid = s.split_wgs > 0 ? s.split_wgs : s.st_nvp;   // virtual planes
            const bool gen = !(s.ldw == s.W && s.st_nsegs == 1);
            s.par_redo = (s.redo && grid_resident(grid, stream_blocks_per_cu(EXACT, ALPHA1, gen, s.st_half != 0))) ? 1 : 0;
            launch_stream(s, dim3(grid), st, EXACT, ALPHA1, gen, s.st_half != 0);
            int rc = launch_check("tv_stream_kernel");
            if (rc) return rc;
            return 0;                    // finalised in-kernel (or main pass only)
        } else {
            const int grid_main = ((P + 7) / 8) * 8 * a.tiles;
            launch_band_main<EXACT, FRONT, ALPHA1>(a, dim3(grid_main), st);
        }
        int rc = launch_check("tv_kernel(main)");
        if (rc) return rc;
    }
    if (!(mask & 2)) return 0;
    // Few workgroups: every one re-derives the per-chain stop flags (cheap) and they meet on one
    // arrival counter -- 8 contending atomics instead of one per CU (measured 13.5 us -> see
    // DESIGN.md).  The rare early-stop recompute is spread over these workgroups.
    const int grid_fin = (P * a.tiles < 8) ? P * a.tiles : 8;
    launch_band_finalise<EXACT, FRONT, ALPHA1>(a, dim3(grid_fin), st);
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
// The fast kernels are compiled for deepinv's TV constants (literal operands, psgla_common.hpp TV_*); a fast request
// with other constants runs the exact kernels (correct at any constants, slower)
static bool tv_fast_constants(const TvArgs& a) {
    return a.tau == TV_TAU && a.opt == TV_OPT && a.sig_tv == TV_SIG && a.rho == TV_RHO && a.inv_opt == TV_INV_OPT;
}

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
    if (d->stream_windows < 0 || d->stream_windows > 2)
        { g_sel_err = "psgla_tv_step: stream_windows must be 0, 1 or 2"; return -1; }
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
        // Shipped tile instances (round 6: none spills a VGPR -- a spill inside a divergent region loses the inactive
        // lanes' values): 32-row tiles (16 waves x 2 rows) always, 48-row tiles (16 x 3) at alpha = 1
        // only; the 72-row tiles (8 x 9) of rounds 4-5 are gone (12-16 chains take the row stream)
        const bool alpha1 = d->x2[0] == nullptr;
        int bh2 = 0, nb2 = 0;
        const int wg3 = alpha1 ? tile_geometry(P, d->H, tile_segs, d->n_tv, 16, 3, &bh, &nb) : 0;
        const int wg2 = tile_geometry(P, d->H, tile_segs, d->n_tv, 16, 2, &bh2, &nb2);
        if (d->kernel_variant == 4 && wg3 == 0 && wg2 == 0) { g_sel_err = "psgla_tv_step: shape not supported by the tile kernel"; return -1; }
        // auto: the tiles fit in one or two rounds on the CUs (measured: castle-size images at B = 3-4 and 321 x 481 at
        // B = 4-6 run faster as two rounds of tiles, profiles/r03l_tile_threshold.txt; since round 6, without the
        // 72-row tiles, 16 chains at 256 x 256 too: 0.0644 vs 0.0680 ms, 12 chains even, profiles/r06m_tile_rounds_ab.txt)
        const long long cus = device_cus();
        const long long ntiles = wg3 > 0 ? (long long)P * nb * tile_segs : (long long)P * nb2 * tile_segs;
        const bool fits2 = wg2 > 0 && (long long)P * nb2 * tile_segs <= cus;
        if ((wg3 > 0 || wg2 > 0) && (d->kernel_variant == 4 || ntiles <= 2 * cus || fits2)) {
            if (wg3 > 0) {
                a.tile_r = 3;
                a.band_h = bh;
                a.nbands = nb;
            } else {
                a.tile_r = 2;
                a.band_h = bh2;
                a.nbands = nb2;
            }
            a.tile_nw = 16;
            // 32-row tiles (2 rows per wave) when they still fit in one round: one or a few images leave most
            // CUs idle at 48 rows (castle B = 1: 114 tiles of 48 rows vs 246 of 32 rows, 41.1 -> 35.0 us,
            // profiles/r03q_tile_r2_ab.txt); more tiles but shorter waves
            if (fits2) {
                a.tile_r = 2;
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
        a.st_half = 0;
        a.st_nvp = d->B * d->C * a.st_nsegs;
        // half windows when they leave fewer lanes idle (castle-like 481 x 321: 2 windows of 256 columns hold
        // 321 -- 63 % of the lanes; 3 half-windows of 128 -- 84 %); stream_windows 1 keeps whole windows
        int hsw = 0;
        const int nh = (a.st_nsegs >= 2 || d->stream_windows == 2) ? stream_segments(a.W, a.ldw, d->n_tv, &hsw, TV_COLS / 2) : 0;
        if (nh > 0 && (d->stream_windows == 2 || (d->stream_windows == 0 &&
            (double)a.W / (nh * (TV_COLS / 2)) > (double)a.W / (a.st_nsegs * TV_COLS) + 0.1))) {
            a.st_half = 1;
            a.st_nsegs = nh;
            a.st_seg_w = hsw;
            a.st_nvp = (d->B * d->C * nh + 1) / 2;
        }
        if (choose_split((long long)a.st_nvp, d->H, d->n_tv, d->stream_wgs, &a.split_wgs)) {
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
    a.redo = d->redo;
    if (d->launch_mask < 0 || d->launch_mask > 4) return fail(0, "psgla_tv_step: launch_mask must be 0 .. 4");
    if (select_step_kernel(d, a) < 0) return g_sel_err == g_err ? (int)hipErrorInvalidValue : fail(0, g_sel_err);
    hipStream_t st = (hipStream_t)stream;
    const int m = d->launch_mask;
    if (d->exact || !tv_fast_constants(a))
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
    return (d->exact || !tv_fast_constants(a)) ? launch_tv<true, FRONT_GIVEN, true>(a, st)
                                               : launch_tv<false, FRONT_GIVEN, true>(a, st);
}

}  // extern "C"

