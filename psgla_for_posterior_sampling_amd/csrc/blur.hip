// Deblurring data term (blur_grad_kernel, blur_sep_kernel) and its C ABI entry point.
// (library overview: psgla_common.hpp)
#include "psgla_common.hpp"

namespace psgla {

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

// One workgroup per (plane, tile), 1-D grid; two resident per CU for l <= 4 (<= 256 VGPRs, 47 KB of LDS).
// Round 6: three per CU (168 VGPRs) spilled 9 VGPRs to scratch, and a VGPR spill inside a divergent (exec-masked)
// region loses the inactive lanes' values -- no shipped kernel spills (tests/test_native_abi.py).
// (A persistent variant that DMA'd the next tile into a second buffer during the passes measured slower:
// two workgroups per CU hide less than three)
#ifndef PSGLA_BLUR_WPE
#define PSGLA_BLUR_WPE 2
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
                    float z[4];   // psgla noise v2: columns j .. j + 3 (j a multiple of 4) are one quad of the row
                    normal_quad(a.seed, (uint32_t)(a.chain0 + tl.b), (uint32_t)step, TAG_LANGEVIN,
                                noise_quad((size_t)tl.c * H + i, j, W), z);
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
            float z[4];   // psgla noise v2: columns j .. j + 3 (j a multiple of 4) are one quad of the row
            normal_quad(a.seed, (uint32_t)(a.chain0 + b), (uint32_t)step, TAG_LANGEVIN, noise_quad((size_t)c * H + i, j, W), z);
            if (vec) {
                const float4 xv = ld4(a.X + o);
                *reinterpret_cast<float4*>(a.Y + o) =
                    make_float4((xv.x + a.c1 * gv[0]) + a.c2 * z[0], (xv.y + a.c1 * gv[1]) + a.c2 * z[1],
                                (xv.z + a.c1 * gv[2]) + a.c2 * z[2], (xv.w + a.c1 * gv[3]) + a.c2 * z[3]);
            } else {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    if (j + kk < W) a.Y[o + kk] = (a.X[o + kk] + a.c1 * gv[kk]) + a.c2 * z[kk];
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

// Fast mode with l >= 7 (15 x 15 and 17 x 17 stencils that are not rank-1: never the reference's kernels, which are)
// takes the exact-order kernel: the fast 2-D instances of those sizes spilled VGPRs to scratch (round 6)
template <bool EXACT>
static void launch_blur(const BlurArgs& a, int l, dim3 grid, hipStream_t st) {
    switch (l) {
#define PSGLA_BLUR_CASE(LL) case LL: hipLaunchKernelGGL((blur_grad_kernel<EXACT, LL>), grid, dim3(BL_THREADS), 0, st, a); break;
#define PSGLA_BLUR_CASE_X(LL) case LL: hipLaunchKernelGGL((blur_grad_kernel<true, LL>), grid, dim3(BL_THREADS), 0, st, a); break;
        PSGLA_BLUR_CASE(0) PSGLA_BLUR_CASE(1) PSGLA_BLUR_CASE(2) PSGLA_BLUR_CASE(3) PSGLA_BLUR_CASE(4)
        PSGLA_BLUR_CASE(5) PSGLA_BLUR_CASE(6) PSGLA_BLUR_CASE_X(7) PSGLA_BLUR_CASE_X(8)
#undef PSGLA_BLUR_CASE_X
#undef PSGLA_BLUR_CASE
        default: break;
    }
}

}  // namespace psgla

using namespace psgla;

extern "C" {

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


}  // extern "C"
