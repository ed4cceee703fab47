/*
 * psgla_hip.h -- C ABI of libpsgla_hip.so, the MI355X (gfx950) hot path of the
 * PSGLA / PnP-ULA Langevin samplers of Marien-RENAUD/PSGLA-for-posterior-sampling.
 *
 * The reference is pure Python: its "interface" for this path is the pair of
 * functions psgla(...) (restoration_algorithms.py:163) and pnpula(...) (:38) plus
 * the closures they call.  Each entry point below replaces a named piece of that
 * loop; the Python host package (psgla_for_posterior_sampling_amd) binds them with
 * ctypes and keeps the reference's signatures (INTEGRATION.md shows the binding a
 * maintainer would add to the reference itself).
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer the caller owns (PyTorch caching allocator);
 *     the library never allocates, frees or synchronises;
 *   - `stream` is a hipStream_t passed as void*; every launch is asynchronous on it,
 *     so the calls are legal inside hipGraph / torch.cuda.graph capture;
 *   - tensors are fp32 NCHW contiguous, one chain per batch entry: (B, C, H, W);
 *     the TV dual is (B, C, H, W, 2) as in deepinv's TVDenoiser;
 *   - the step index i of the Langevin loop is read from `*d_step + step_offset`
 *     when d_step != NULL (device counter, for graph replay), else it is
 *     `step_offset`;
 *   - return 0 on success or a hipError_t value; psgla_last_error() describes the
 *     last failure of the calling thread.  Nothing throws across the ABI.
 */
#ifndef PSGLA_HIP_H_
#define PSGLA_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSGLA_HIP_ABI_VERSION 11

/* Max inner TV iterations the fused (temporally blocked) kernel handles. */
#define PSGLA_TV_MAX_FUSED_IT 24

int psgla_abi_version(void);
const char* psgla_last_error(void);

/* ---------------------------------------------------------------------------------
 * Sample storage and running mean / second moment
 *   reference: restoration_algorithms.py:240-244 (samples every n_inter steps) and
 *   :255-271 (online block means of X and X^2; a block holds n_inter_mmse+1 samples,
 *   the trailing partial block is dropped).  Step i uses acc_coef[i mod (nm+1)] =
 *   (fp32(k/(k+1)), fp32(1/(k+1))); the block index is i / (nm+1).
 * ------------------------------------------------------------------------------- */
typedef struct PsglaSchedule {
    int64_t* d_step;          /* device step counter, or NULL (then step_offset is the step) */
    int64_t step_offset;
    int32_t n_inter;          /* X stored when i % n_inter == 0; <= 0: never            */
    int32_t n_inter_mmse;     /* < 0: no accumulation                                    */
    const float* acc_coef;    /* device [(n_inter_mmse+1) * 2]                           */
    float* samples;           /* [samples_cap][B][C][H][W] or NULL                       */
    int64_t samples_cap;
    float* blocks;            /* [blocks_cap][B][C][H][W] block means of X               */
    float* blocks2;           /* [blocks_cap][B][C][H][W] block means of X^2             */
    int64_t blocks_cap;
} PsglaSchedule;

/* ---------------------------------------------------------------------------------
 * psgla_tv_step: ONE fused PSGLA Langevin step with the inpainting fidelity and the
 * warm-started TV prox, for B chains.  Replaces one iteration of
 *   restoration_algorithms.py:231-271 with
 *   data_grad = sampling_images.py:295  (-mask*(x - y)/sigma2)
 *   denoiser  = deepinv 0.2.1 TVDenoiser(n_it_max) (sampling_images.py:138), ths = s
 * i.e.  Z ~ N(0,1);  Y = (X + c1*g(X)) + c2*Z;  X' = (1-alpha)*Y + alpha*TVprox(Y);
 *       accumulators / samples per PsglaSchedule.
 * State is double-buffered by step parity: step i reads x[i&1], u2[i&1], ...
 * and writes x[(i+1)&1], ...  deepinv's early stop (rel_err < tol at inner iteration
 * k >= 2, per chain: the affected chains are recomputed with k+1 inner iterations)
 * is honoured, `fresh` is cleared and *d_step advanced once the step is complete.
 * What is launched depends on the variant the shape selects (kernel_variant 0):
 *   - the small-batch tile kernel (tv_tile_kernel: any W, rows padded to the pitch ldw and cut
 *     into the stream kernel's column segments when W > 256) when its 32-, 48- or 72-row tiles
 *     all fit on the CUs at once (few chains per GPU, or a few real-size images; two rounds of
 *     48-row tiles for segmented rows): ONE launch of at most 32767 tiles; its last workgroup
 *     to arrive evaluates the early stop, recomputes stopped chains and advances the step (no
 *     second kernel);
 *   - else the row-streaming kernel (tv_stream_kernel: row pitch ldw % 4 == 0,
 *     1 <= n_tv <= 10, H >= 2, every width with column segments, any alpha): one row per
 *     pipeline step, ONE launch, finalised in-kernel;
 *   - otherwise (n_tv > 10 or H < 2, or kernel_variant 1) the temporally blocked
 *     band kernel (tv_main_kernel) followed by a small finaliser kernel
 *     (tv_finalise_kernel, <= 8 workgroups) that does the same.
 * launch_mask 1 launches only the main pass of either variant (timing).
 * deepinv's early stop (rare at the reference's settings) in the row stream and the tile kernel with a `redo`
 * buffer (ABI 11) and a grid the CUs hold at once: the step's finaliser only records which chains stopped
 * (redo[4 + g] = their inner-iteration count, redo[0] = pending); the NEXT launch's workgroups first redo the
 * stopped chains' part of that step -- every workgroup its own rows / tile, all in parallel --, meet at one grid
 * barrier (redo[1]), then run their own step.  A run's last step is settled by launch_mask 4 (the pending redo
 * alone, then redo[0] cleared), which the host issues before it reads results.  Without `redo` (or with a larger
 * grid), the finaliser's workgroup recomputes the stopped chains itself, one (plane, segment) / tile after another.
 * ------------------------------------------------------------------------------- */
typedef struct PsglaTvStep {
    int32_t B, C, H, W;
    float* x[2];              /* chain state X (B,C,H,W)                                */
    float* u2[2];             /* TV dual (B,C,H,W,2)                                    */
    float* x2[2];             /* TV primal when alpha != 1; NULL when alpha == 1 (x2==X)*/
    float* mean[2];           /* live block accumulators (B,C,H,W); NULL if no accum    */
    float* sq[2];
    const float* y;           /* observation (B,C,H,W); chain stride y_chain_stride     */
    int64_t y_chain_stride;   /* elements; 0 = one observation shared by all chains     */
    const uint8_t* mask;      /* inpainting mask (H,W) per chain, 1 = observed          */
    int64_t mask_chain_stride;/* bytes; 0 = shared                                       */
    float c1;                 /* fp32(delta)/fp32(lambd)    (restoration_algorithms.py:236) */
    float c2;                 /* fp32(sqrt 2) * fp32(s)     (:228, :236)                  */
    float sigma2;             /* fp32(sigma1^2), used as a divisor (sampling_images.py:295) */
    float alpha;              /* relaxation (:238)                                        */
    float tau, one_plus_tau, sigma_tv, rho, ths, tol;  /* TVDenoiser constants (fp32)     */
    int32_t n_tv;             /* inner iterations n_it_max (<= PSGLA_TV_MAX_FUSED_IT)     */
    int32_t exact;            /* 1: reference op order + IEEE div/sqrt (bit-exact checker mode);
                                 0 (fast) runs the fast kernels only for deepinv's TV constants
                                 (tau 0.01, rho 1.99, sigma 1/(8 tau) in fp32): others take the exact ones */
    uint64_t seed;            /* seed_alg                                                 */
    int32_t chain0;           /* global id of chain 0 of this batch (multi-GPU sharding)  */
    int32_t advance_step;     /* 1: finaliser increments *d_step                           */
    int32_t* fresh;           /* device int: 1 -> TV restart (x2=Y, u2=0), cleared after the step */
    double* norms;            /* device [B][n_tv][2], zero-initialised (rel_err partial sums) */
    int32_t* arrive;          /* device int[4], zero-initialised: [0] finaliser arrival counter (zero
                                 again once each step's launch has completed); [3] (ABI 9) set to 1
                                 if the tile kernel's early-stop recompute ever stopped waiting for
                                 the other workgroups' stores (a guard that should never expire:
                                 the host checks it, FusedTvChains.check_handoff)               */
    int32_t launch_mask;      /* 0 or 3: both kernels; 1: tile kernel only (re-runs the same step:
                                 idempotent, for kernel timing); 2: finaliser only; 4 (ABI 11): settle a
                                 pending early-stop redo of the last step (no step is run)     */
    int32_t kernel_variant;   /* 0: auto (see above); 1: force the band kernel; 2: force the row stream
                                 (one row per pipeline step); 4: force the small-batch tile kernel
                                 (ldw % 4 == 0).  Other values (3 included: the row-pair pipeline
                                 of ABI 6 is gone) are rejected. */
    int32_t stream_wgs;       /* streaming kernel work split: 0 auto (rows of all planes cut into
                                 one contiguous range per CU, n_tv halo rows at cuts, when W <= 256);
                                 -1 one workgroup per plane; > 0 force that many row ranges      */
    int32_t ldw;              /* row pitch (elements) of every (.., H, W) buffer: x, u2 (x2 per
                                 element pair), x2, mean, sq, y, mask, samples, blocks; 0 = W.
                                 ldw != W (a multiple of 4 >= W: rows padded so that W % 4 != 0
                                 images run on the streaming / tile kernels) needs one of them;
                                 the padding columns are scratch (never read into the image).
                                 The noise stream is indexed by the unpadded element.            */
    int32_t norms_copies;     /* (ABI 8) 0 or 1: norms is [B][n_tv][2]; K > 1: norms holds K zero-initialised
                                 copies [K][B][n_tv][2] and the tile kernel spreads its workgroups'
                                 rel-err partial sums over them (workgroup x adds to copy x % K), so
                                 that many tiles of one chain do not queue on the same atomics   */
    int32_t stream_windows;   /* (ABI 9) row-stream column windows: 0 auto (256 < W <= 324 at n_tv = 10:
                                 half-wave windows, two 128-column segments per wave, where whole
                                 256-column windows would leave a third of the lanes idle); 1 whole
                                 256-column windows only; 2 half-wave windows whenever they fit
                                 (diagnostic: the halo cost of 128-column pipelines at any width)  */
    int32_t* redo;            /* (ABI 11) device int[4 + B], zero-initialised, or NULL: the parallel early-stop
                                 redo (above): [0] pending (bit 0) and the stopped step's TV restart flag
                                 (bit 1), [1] the grid-barrier count, [4 + g] chain g's inner iterations  */
} PsglaTvStep;

int psgla_tv_step(const PsglaTvStep* d, const PsglaSchedule* s, void* stream);
/* Which kernel psgla_tv_step launches for this descriptor (host-side query, launches nothing):
 * 0 band kernel + finaliser, 1 row stream (tv_stream_kernel), 3 small-batch tile kernel
 * (tv_tile_kernel); -1 if the descriptor is rejected.  (2 is unused since ABI 7.) */
int psgla_tv_step_kernel(const PsglaTvStep* d);

/* ---------------------------------------------------------------------------------
 * psgla_tv_prox: TVDenoiser.forward(y, ths) on a (B,C,H,W) tensor, deepinv 0.2.1
 * semantics: warm start from (x2_in, u2_in) unless `fresh`; early stop on the
 * relative change of the WHOLE tensor (as deepinv computes it), or of each chain
 * (per_chain = 1: B independent reference runs, psgla's loop over a chain batch).
 * Outputs x2_out, u2_out (new buffers, like deepinv's out-of-place updates).
 * One call runs n_tv <= PSGLA_TV_MAX_FUSED_IT inner iterations; a longer
 * n_it_max runs as consecutive calls ("chunks", hip_ops.tv_prox): chunk c has
 * it0 = the global index of its first iteration (deepinv tests rel_err from
 * global iteration 2 on), last_chunk = 1 on the final one, and reports in
 * stopped[g] (device, [groups]) the iteration count after which group g stopped
 * inside the chunk (0: it did not stop); the host then keeps that group's result.
 * ------------------------------------------------------------------------------- */
typedef struct PsglaTvProx {
    int32_t B, C, H, W;
    const float* y;
    const float* x2_in;  const float* u2_in;   /* ignored when fresh                      */
    float* x2_out;       float* u2_out;
    float tau, one_plus_tau, sigma_tv, rho, ths, tol;
    int32_t n_tv, exact, fresh;
    double* norms;            /* device [groups][n_tv][2], zeroed (groups = B if per_chain else 1) */
    int32_t* arrive;          /* device int, zeroed       */
    int32_t per_chain;        /* 1: early stop per chain (batch of independent chains)           */
    int32_t it0;              /* global index of this call's first inner iteration (0 = whole call) */
    int32_t last_chunk;       /* 1 (default use): no further chunk follows                         */
    int32_t* stopped;         /* device [groups] or NULL: stop count inside this chunk, 0 = none   */
} PsglaTvProx;

int psgla_tv_prox(const PsglaTvProx* d, void* stream);

/* ---------------------------------------------------------------------------------
 * Generic (opaque-closure) building blocks.
 * ------------------------------------------------------------------------------- */
/* out[b][e] = N(0,1) of "psgla noise v2" (seed, chain0+b, step, tag);  torch.randn at
 * restoration_algorithms.py:232 / :104.  A chain's E elements are rows of W (the image width:
 * E = C*H*W); noise quads never straddle two rows (psgla_for_posterior_sampling_amd/csrc/noise.hpp).
 * (ABI 10: W added; ABI <= 9 numbered the quads over the flat index, which differs for W % 4 != 0.) */
int psgla_normal_fill(float* out, int32_t B, int64_t E, int32_t W, uint64_t seed, int32_t chain0,
                      const int64_t* d_step, int64_t step_offset, uint32_t tag, void* stream);

/* Y = (X + c1*g) + c2*Z  (restoration_algorithms.py:232-236); E = C*H*W elements per chain in rows of W */
int psgla_langevin_update(const float* X, const float* g, float* Y, int32_t B, int64_t E, int32_t W, float c1,
                          float c2, uint64_t seed, int32_t chain0, const int64_t* d_step,
                          int64_t step_offset, void* stream);

/* X = (1-alpha)*Y + alpha*D, then samples / block accumulators (restoration_algorithms.py:238-271).
 * mean/sq are (B,C,H,W) live accumulators updated in place. */
int psgla_relax_accumulate(const float* Y, const float* D, float* X, float alpha, int32_t alpha_is_one,
                           float* mean, float* sq, int32_t B, int64_t E, const PsglaSchedule* s,
                           void* stream);

/* DNN-denoiser PSGLA, inpainting: the epilogue of step i fused with the prologue of step i+1
 * (restoration_algorithms.py:238-271 then :232-236 with sampling_images.py:295):
 *   X = (1-alpha)*Y + alpha*D  (X = D when alpha_is_one; Y may then be NULL);
 *   samples / block accumulators of step i (PsglaSchedule, as psgla_relax_accumulate);
 *   Y_next = (X + c1*g(X)) + c2*Z_{i+1},  g = ((-m)*(X - y))/sigma2,  Z_{i+1} the noise of step i+1;
 *   X is stored only when X != NULL.  Any H, W (W % 4 != 0: a scalar variant over the chain's
 *   row-aligned noise quads, as psgla_langevin_update).  Identical to psgla_relax_accumulate +
 *   psgla_inpaint_grad + psgla_langevin_update, in one pass (28 B/elem at alpha = 1). */
int psgla_relax_langevin_inpaint(const float* Y, const float* D, float* X, float alpha, int32_t alpha_is_one,
                                 const float* y, int64_t y_chain_stride, const uint8_t* mask,
                                 int64_t mask_chain_stride, float* Y_next, float* mean, float* sq, int32_t B,
                                 int32_t C, int32_t H, int32_t W, float sigma2, float c1, float c2, uint64_t seed,
                                 int32_t chain0, const PsglaSchedule* s, void* stream);

/* PnP-ULA update (restoration_algorithms.py:104-115) + samples / accumulators:
 *   proj = clip(X, c_min, c_max); X' = (X + delta*((gp - (X-proj)/lambd) + gd)) + brw*Z */
int pnpula_update(const float* X, const float* gp, const float* gd, float* Xout, float delta,
                  float lambd, float brw, float c_min, float c_max, float* mean, float* sq,
                  int32_t B, int64_t E, int32_t W, uint64_t seed, int32_t chain0, const PsglaSchedule* s,
                  void* stream);

/* PnP-ULA step with the DNN prior fused ("V-ULA"): replaces, in one pass over the chain state,
 *   gp = (alpha * (D - X)) / s2             DenoiserPrior, sampling_images.py:156-157 (D = D(X, s1))
 *   gd = ((-m) * (X - y)) / sigma2          sampling_images.py:295, when gd == NULL (inpainting;
 *                                           y / mask as psgla_inpaint_grad), else the given gd
 *                                           (deblurring: psgla_blur_grad's output)
 *   the update of pnpula_update (restoration_algorithms.py:104-115) and its accumulators.
 * Same fp32 operations in the same order as those three steps (bit-identical); 32 B/elem at
 * inpainting (read X, D, y, mean, sq; write X', mean, sq).  X, D, Xout: (B, C, H, W). */
int pnpula_prior_update(const float* X, const float* D, float alpha, float s2, const float* gd, const float* y,
                        int64_t y_chain_stride, const uint8_t* mask, int64_t mask_chain_stride, float sigma2,
                        float* Xout, float delta, float lambd, float brw, float c_min, float c_max, float* mean,
                        float* sq, int32_t B, int32_t C, int32_t H, int32_t W, uint64_t seed, int32_t chain0,
                        const PsglaSchedule* s, void* stream);
/* g = ((-m) * (X - y)) / sigma2, mask (H,W) u8 per chain (sampling_images.py:295) */
int psgla_inpaint_grad(const float* X, const float* y, int64_t y_chain_stride, const uint8_t* mask,
                       int64_t mask_chain_stride, float* g, int32_t B, int32_t C, int32_t H,
                       int32_t W, float sigma2, void* stream);

/* Deblurring data term (sampling_images.py:329-338), circular (2l+1)^2 depthwise stencils:
 *   g = -A^T(A X - y) / sigma2,  A = conv2d(pad(., l, circular), hconv),  A^T: same with hcorr
 * hconv / hcorr: HOST arrays of (2l+1)^2 fp32 taps (row-major, the same for every channel;
 *   copied into the launch's arguments), l <= 8.  X, y, g, Y: device.
 * With Y != NULL the Langevin update of restoration_algorithms.py:232-236 is fused:
 *   Y = (X + c1 g) + c2 Z  (Z: the noise stream of psgla_langevin_update) and g is not written;
 * else g is written.  exact = 1: multiply-then-add taps and IEEE division (else fma, 1/sigma2). */
int psgla_blur_grad(const float* X, const float* y, int64_t y_chain_stride, const float* hconv, const float* hcorr,
                    int32_t l, float* g, float* Y, int32_t B, int32_t C, int32_t H, int32_t W, float sigma2,
                    float c1, float c2, uint64_t seed, int32_t chain0, const int64_t* d_step, int64_t step_offset,
                    int32_t exact, void* stream);
/* Fast mode (exact = 0) runs rank-1 taps (the reference's h^T h kernels) as separable row / column passes
 * (results within fp32 rounding of the 2-D stencil); enable = 0 keeps every call on the 2-D stencil
 * (process-wide switch, for A/B and tests; default 1). */
int psgla_blur_set_separable(int32_t enable);
/* *d_step += 1 (one thread) */
int psgla_advance_step(int64_t* d_step, void* stream);

/* DnCNN conv epilogue (the deepinv DnCNN the reference loads, sampling_images.py:129-134, called at
 * restoration_algorithms.py:238): y = relu(y + bias[c]) (relu != 0) or y + bias[c], in place, n
 * elements.  Layout NHWC when hw == 0 (channel fastest, C % 4 == 0), NCHW with plane size hw
 * (hw % 4 == 0) otherwise.  Same fp32 operations as PyTorch's bias add + clamp_min(0). */
int psgla_bias_act(float* y, const float* bias, int64_t n, int32_t C, int64_t hw, int32_t relu, void* stream);

/* Diagnostic (tests): Box-Muller radius r(k) and (cos, sin)(2 pi k 2^-24) of the noise stream for the
 * 24-bit indices k0 .. k0+n-1, so the GPU stream can be checked against the CPU checker exhaustively. */
int psgla_debug_bm_tables(float* r, float* cs, float* sn, uint32_t k0, uint32_t n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PSGLA_HIP_H_ */
