"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the golden
fixtures made by the reference itself.  Bit-exact where the kernel runs in EXACT mode or
the op is integer / elementwise; the north-star tolerance (1e-5 relative, fp32, on the
sample mean) for the fast TV kernels."""
import os

import numpy as np
import pytest
import torch

from oracle import psgla_oracle as orc

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda:0"

# north-star tolerance on the sample mean (fp32): ||a - b|| / ||b|| <= 1e-5
REL_TOL_MEAN = 1e-5


def load(name):
    return dict(np.load(os.path.join(G, name + ".npz"), allow_pickle=False))


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from psgla_for_posterior_sampling_amd import _native as N
    N.lib()
    yield


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


# ------------------------------------------------------------------------------ noise
def test_noise_tables_exhaustive():
    """All 2^24 Box-Muller radii and all 2^24 angles: GPU == CPU checker, bit for bit."""
    import ctypes
    from psgla_for_posterior_sampling_amd import _native as N
    n = 1 << 24
    r = torch.empty(n, device=DEV)
    c = torch.empty(n, device=DEV)
    s = torch.empty(n, device=DEV)
    N.check(N.lib().psgla_debug_bm_tables(r.data_ptr(), c.data_ptr(), s.data_ptr(), 0, n,
                                          torch.cuda.current_stream().cuda_stream), "bm_tables")
    torch.cuda.synchronize()
    rr = orc.radius_table(0, n)
    cc, ss = orc.angle_table(0, n)
    np.testing.assert_array_equal(r.cpu().numpy(), rr)
    np.testing.assert_array_equal(c.cpu().numpy(), cc)
    np.testing.assert_array_equal(s.cpu().numpy(), ss)


@pytest.mark.parametrize("shape,seed,chain0,step", [((1, 3, 24, 40), 0, 0, 0), ((3, 3, 17, 31), 5, 7, 123),
                                                     ((2, 1, 5, 7), 2 ** 40 + 3, 0, 99999)])
def test_normal_fill_matches_checker(shape, seed, chain0, step):
    from psgla_for_posterior_sampling_amd import hip_ops as K
    out = torch.empty(shape, device=DEV)
    K.normal_fill(out, seed, chain0, step)
    got = out.cpu()
    for b in range(shape[0]):
        ref = orc.normal((1,) + shape[1:], seed, chain0 + b, step)
        assert torch.equal(got[b:b + 1], ref)


# ------------------------------------------------------------------------------ TV prox
def _tv_case(shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    y = torch.rand(shape, generator=g) + 0.05 * torch.randn(shape, generator=g)
    return y


@pytest.mark.parametrize("shape", [(1, 3, 24, 40), (2, 3, 70, 300), (1, 1, 5, 7), (1, 3, 33, 321)])
@pytest.mark.parametrize("n_it", [10, 3])
def test_tv_prox_exact_bitwise(shape, n_it):
    from psgla_for_posterior_sampling_amd.denoisers import TVDenoiser
    y = _tv_case(shape)
    ths = torch.tensor(10 / 255.0, dtype=torch.float32)
    ref = orc.TVDenoiser(n_it_max=n_it)
    gpu = TVDenoiser(n_it_max=n_it, exact=True)
    for call in range(3):   # first call restarts, later calls warm-start
        yy = y + 0.01 * call
        out_ref = ref.forward(yy, ths)
        out = gpu.forward(yy.to(DEV), ths)
        np.testing.assert_array_equal(out.cpu().numpy(), out_ref.numpy(), err_msg=f"call {call}")
        np.testing.assert_array_equal(gpu.u2.cpu().numpy(), ref.u2.numpy())


def test_tv_prox_early_stop_exact():
    """tol large enough that deepinv's early stop fires: the finaliser must redo with k+1 its."""
    from psgla_for_posterior_sampling_amd.denoisers import TVDenoiser
    y = _tv_case((1, 3, 40, 52), seed=3)
    ths = torch.tensor(10 / 255.0, dtype=torch.float32)
    ref = orc.TVDenoiser(n_it_max=10, tol=3e-2)
    gpu = TVDenoiser(n_it_max=10, tol=3e-2, exact=True)
    out_ref = ref.forward(y, ths)
    assert ref.last_n_it < 10, "test needs the early stop to fire"
    out = gpu.forward(y.to(DEV), ths)
    np.testing.assert_array_equal(out.cpu().numpy(), out_ref.numpy())


@pytest.mark.parametrize("shape", [(1, 3, 24, 40), (2, 3, 130, 260)])
def test_tv_prox_fast_tolerance(shape):
    from psgla_for_posterior_sampling_amd.denoisers import TVDenoiser
    y = _tv_case(shape, seed=1)
    ths = torch.tensor(10 / 255.0, dtype=torch.float32)
    ref = orc.TVDenoiser(n_it_max=10)
    gpu = TVDenoiser(n_it_max=10, exact=False)
    for call in range(3):
        out_ref = ref.forward(y, ths)
        out = gpu.forward(y.to(DEV), ths)
        assert rel(out.cpu().numpy(), out_ref.numpy()) < 5e-6
        assert np.abs(out.cpu().numpy() - out_ref.numpy()).max() < 1e-5


# ------------------------------------------------------------------------------ fused PSGLA + TV
def _run_fused_vs_fixture(exact):
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.denoisers import TVDenoiser
    from psgla_for_posterior_sampling_amd.fidelity import InpaintingFidelity
    fx = load("psgla_inpaint_tv")
    seed, n, ni, nm, alpha, lam, s, delta, ntv = fx["meta"]
    y = torch.from_numpy(fx["y"]).to(DEV)
    mask = torch.from_numpy(fx["mask2d"]).to(DEV)
    sigma2 = torch.tensor((1 / 255.0) ** 2, dtype=torch.float32)
    dg = InpaintingFidelity(mask, y, sigma2)
    tv = TVDenoiser(n_it_max=int(ntv), exact=exact)
    out = RA.psgla(torch.from_numpy(fx["init"]).to(DEV), dg, tv, torch.tensor(alpha, dtype=torch.float32),
                   torch.tensor(lam, dtype=torch.float32), sig_float=float(s), delta=float(delta),
                   n_iter=int(n), n_inter=int(ni), n_inter_mmse=int(nm), seed=int(seed), graph_steps=20)
    Xl, Ml, M2l = [np.stack([t.cpu().numpy() for t in lst]) for lst in out]
    return fx, Xl, Ml, M2l, tv


def test_fused_psgla_tv_exact_matches_reference_fixture():
    fx, Xl, Ml, M2l, tv = _run_fused_vs_fixture(exact=True)
    np.testing.assert_array_equal(Xl, fx["samples"])
    np.testing.assert_array_equal(Ml, fx["blocks"])
    np.testing.assert_array_equal(M2l, fx["blocks2"])
    np.testing.assert_array_equal(tv.x2.cpu().numpy(), fx["tv_x2"])
    np.testing.assert_array_equal(tv.u2.cpu().numpy(), fx["tv_u2"])


def test_fused_psgla_tv_postprocessing_matches_reference():
    """The CLI's per-image record (metrics.analyse_run over psgla's lists, as restore_image runs it)
    against sampling_images.py:371-442 executed by the reference's own code on the reference's own
    chain outputs (tests/golden/postproc_inpaint_tv.npz): identical, since the exact kernel's lists
    are bit-identical to the fixture's."""
    from psgla_for_posterior_sampling_amd import metrics
    fx, Xl, Ml, M2l, tv = _run_fused_vs_fixture(exact=True)
    ref = load("postproc_inpaint_tv")
    im = np.float32(np.transpose(fx["x"][0], (1, 2, 0)))
    to = lambda a: [torch.from_numpy(t) for t in a]   # noqa: E731
    rec, _ = metrics.analyse_run(im, to(Xl), to(Ml), to(M2l), torch.from_numpy(fx["y"]),
                                 torch.from_numpy(fx["init"]))
    for k in ("PSNR_sample", "SIM_sample", "PSNR_mmse", "SIM_list"):
        np.testing.assert_allclose(np.array(rec[k]), ref[k], rtol=1e-6, atol=0, err_msg=k)
    for k in ("PSNR_MMSE", "SIM_MMSE", "PSNR_y"):
        assert abs(rec[k] - float(ref[k])) <= 1e-6 * abs(float(ref[k])), k
    for k in ("MMSE", "std", "diff"):
        np.testing.assert_allclose(rec[k], ref[k], rtol=0, atol=1e-6, err_msg=k)


def test_fused_psgla_tv_fast_within_tolerance():
    fx, Xl, Ml, M2l, tv = _run_fused_vs_fixture(exact=False)
    assert rel(Ml.mean(0), fx["blocks"].mean(0)) < REL_TOL_MEAN
    assert rel(M2l.mean(0), fx["blocks2"].mean(0)) < REL_TOL_MEAN
    assert Xl.shape == fx["samples"].shape


def _fused_batch(B, chain0, exact, n_iter=40, H=48, W=64, alpha=1.0, variant="auto", stream_wgs=0, n_inter=5,
                 n_inter_mmse=4):
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator().manual_seed(5)
    x = torch.rand((1, 3, H, W), generator=g)
    dg, y, init, mask2d = orc.inpainting_problem(x, seed_ip=1)
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    eng = FusedTvChains(init.expand(B, -1, -1, -1).contiguous().to(DEV), y.to(DEV),
                        mask2d.to(torch.uint8).to(DEV), c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)),
                        alpha=alpha, ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=10), seed=3,
                        n_iter=n_iter, n_inter=n_inter, n_inter_mmse=n_inter_mmse, chain0=chain0, exact=exact,
                        kernel_variant=variant, stream_wgs=stream_wgs)
    return eng, (dg, y, init, mask2d, c1, c2)


@pytest.mark.parametrize("variant", ["stream", "band", "tile"])
def test_fused_chains_independent_of_batching_and_graph(variant):
    """Chain k's trajectory depends only on (seed, global chain id): B=4 batch vs B=2 batch
    with chain0=2, and eager vs hipGraph replay -- bit-identical (multi-GPU sharding property)."""
    e4, _ = _fused_batch(4, 0, exact=False, variant=variant)
    e4.run(40, graph_steps=0)
    e2, _ = _fused_batch(2, 2, exact=False, variant=variant)
    e2.run(40, graph_steps=10)
    torch.cuda.synchronize()
    assert torch.equal(e4.X[2:], e2.X)
    b4, _ = e4.blocks()
    b2, _ = e2.blocks()
    assert torch.equal(b4[:, 2:], b2)
    assert torch.equal(e4.samples()[:, 2:], e2.samples())


@pytest.mark.parametrize("variant,H,W", [("stream", 48, 64), ("band", 48, 64), ("stream", 70, 300),
                                          ("band", 70, 300), ("auto", 37, 29)])
def test_fused_multichain_exact_vs_oracle(variant, H, W):
    B = 3
    eng, (dg, y, init, mask2d, c1, c2) = _fused_batch(B, 10, exact=True, n_iter=30, H=H, W=W, variant=variant)
    eng.run(30, graph_steps=0)
    torch.cuda.synchronize()
    for b in range(B):
        tv = orc.TVDenoiser(n_it_max=10)
        Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(1.0), torch.tensor(10.0), sig_float=10 / 255.0,
                                delta=(10 / 255.0) ** 2, n_iter=30, n_inter=5, n_inter_mmse=4, seed=3,
                                chain=10 + b)
        np.testing.assert_array_equal(eng.samples()[:, b].cpu().numpy(), np.stack([t.numpy() for t in Xl]))
        bm, bm2 = eng.blocks()
        np.testing.assert_array_equal(bm[:, b].cpu().numpy(), np.stack([t.numpy() for t in Ml]))
        np.testing.assert_array_equal(bm2[:, b].cpu().numpy(), np.stack([t.numpy() for t in M2l]))


_ORACLE_CACHE = {}


def _oracle_chain(init, dg, n_iter, chain):
    key = (n_iter, chain, tuple(init.shape))
    if key not in _ORACLE_CACHE:
        tv = orc.TVDenoiser(n_it_max=10)
        Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(1.0), torch.tensor(10.0), sig_float=10 / 255.0,
                                delta=(10 / 255.0) ** 2, n_iter=n_iter, n_inter=5, n_inter_mmse=4, seed=3,
                                chain=chain)
        _ORACLE_CACHE[key] = (np.stack([t.numpy() for t in Xl]), np.stack([t.numpy() for t in Ml]),
                              np.stack([t.numpy() for t in M2l]), tv.x2.numpy(), tv.u2.numpy())
    return _ORACLE_CACHE[key]


@pytest.mark.parametrize("variant", ["stream"])
@pytest.mark.parametrize("stream_wgs", [-1, 3, 4, 7, 11, 20, 97])
def test_stream_row_split_exact_vs_oracle(stream_wgs, variant):
    """Row-split streaming (the plane rows of all chains cut into stream_wgs ranges, n_tv halo rows
    at cuts inside a plane, ranges spanning plane boundaries): bit-identical to the checker for every cut position; -1 = one workgroup per plane."""
    B, H, W, n_iter = 3, 48, 64, 20
    eng, (dg, y, init, mask2d, c1, c2) = _fused_batch(B, 10, exact=True, n_iter=n_iter, H=H, W=W,
                                                      variant=variant, stream_wgs=stream_wgs)
    assert eng.main_kernel == "tv_stream_kernel"
    eng.run(n_iter, graph_steps=0)
    torch.cuda.synchronize()
    bm, bm2 = eng.blocks()
    for b in range(B):
        Xs, Ms, M2s, x2, u2 = _oracle_chain(init, dg, n_iter, 10 + b)
        np.testing.assert_array_equal(eng.samples()[:, b].cpu().numpy(), Xs)
        np.testing.assert_array_equal(bm[:, b].cpu().numpy(), Ms)
        np.testing.assert_array_equal(bm2[:, b].cpu().numpy(), M2s)
        np.testing.assert_array_equal(eng.u2_state[b].cpu().numpy(), u2[0])


class _RecordingTV(orc.TVDenoiser):
    def __init__(self, **kw):
        super().__init__(**kw)
        self.its = []

    def forward(self, y, ths):
        out = super().forward(y, ths)
        self.its.append(self.last_n_it)
        return out


@pytest.mark.parametrize("variant", ["stream"])
@pytest.mark.parametrize("stream_wgs", [0, -1])
def test_stream_early_stop_exact_vs_oracle(stream_wgs, variant):
    """tol large enough that deepinv's early stop fires in some steps: the stream kernel's last
    workgroup re-streams the stopped chains' planes with k+1 iterations -- bit-identical."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    B, H, W, n_iter, tol = 2, 40, 52, 12, 3e-2
    g = torch.Generator().manual_seed(7)
    x = torch.rand((1, 3, H, W), generator=g)
    dg, y, init, mask2d = orc.inpainting_problem(x, seed_ip=2)
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    eng = FusedTvChains(init.expand(B, -1, -1, -1).contiguous().to(DEV), y.to(DEV), mask2d.to(torch.uint8).to(DEV),
                        c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)), alpha=1.0,
                        ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=10, tol=tol), seed=4,
                        n_iter=n_iter, n_inter=3, n_inter_mmse=2, exact=True, kernel_variant=variant,
                        stream_wgs=stream_wgs)
    eng.run(n_iter, graph_steps=0)
    torch.cuda.synchronize()
    bm, bm2 = eng.blocks()
    fired = False
    for b in range(B):
        tv = _RecordingTV(n_it_max=10, tol=tol)
        Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(1.0), torch.tensor(10.0), sig_float=10 / 255.0,
                                delta=(10 / 255.0) ** 2, n_iter=n_iter, n_inter=3, n_inter_mmse=2, seed=4, chain=b)
        fired = fired or min(tv.its) < 10
        np.testing.assert_array_equal(eng.samples()[:, b].cpu().numpy(), np.stack([t.numpy() for t in Xl]))
        np.testing.assert_array_equal(bm[:, b].cpu().numpy(), np.stack([t.numpy() for t in Ml]))
        np.testing.assert_array_equal(eng.u2_state[b].cpu().numpy(), tv.u2.numpy()[0])
    assert fired, "test needs the early stop to fire"


def test_stream_row_split_rejects_bad_counts():
    from psgla_for_posterior_sampling_amd._native import NativeLibraryError
    for bad in (1, 10 ** 6):           # fewer than ceil(B*C/3) ranges / more ranges than rows
        with pytest.raises((RuntimeError, NativeLibraryError)):
            eng, _ = _fused_batch(3, 0, exact=True, n_iter=10, variant="stream", stream_wgs=bad)
            eng.run(1, graph_steps=0)
            torch.cuda.synchronize()


@pytest.mark.parametrize("variant", ["stream", "band"])
def test_fused_alpha_not_one_exact_vs_oracle(variant):
    eng, (dg, y, init, mask2d, c1, c2) = _fused_batch(1, 0, exact=True, n_iter=20, alpha=0.6, variant=variant)
    eng.run(20)
    torch.cuda.synchronize()
    tv = orc.TVDenoiser(n_it_max=10)
    Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(0.6), torch.tensor(10.0), sig_float=10 / 255.0,
                            delta=(10 / 255.0) ** 2, n_iter=20, n_inter=5, n_inter_mmse=4, seed=3, chain=0)
    np.testing.assert_array_equal(eng.samples()[:, 0].cpu().numpy(), np.stack([t.numpy() for t in Xl]))
    np.testing.assert_array_equal(eng.x2_state.cpu().numpy(), tv.x2.numpy())


def test_fused_full_size_fast_vs_exact():
    """BASELINE size (64 chains x 3x256x256), a few steps: fast vs exact kernels agree to fp32
    rounding, no NaN, and the per-chain state stays bounded."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator(device=DEV).manual_seed(1234)
    x = torch.rand((1, 3, 256, 256), generator=g, device=DEV)
    from psgla_for_posterior_sampling_amd.fidelity import inpainting_problem
    dg, y, init, mask2d, _ = inpainting_problem(x)
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    outs = []
    for exact, variant in ((True, "stream"), (False, "stream"), (True, "band")):
        eng = FusedTvChains(init.expand(64, -1, -1, -1).contiguous(), y, dg.mask_u8, c1=c1, c2=c2,
                            sigma2=dg.sigma2, alpha=1.0, ths=float(np.float32(10 / 255.0)),
                            tv=K.TvConstants(n_it_max=10), seed=0, n_iter=12, n_inter=10, n_inter_mmse=10,
                            exact=exact, kernel_variant=variant)
        eng.run(12, graph_steps=0)
        torch.cuda.synchronize()
        outs.append((eng.X.clone(), eng.blocks()[0].clone()))
    (xe, be), (xf, bf), (xb, bb) = outs
    assert torch.equal(xe, xb) and torch.equal(be, bb)      # the exact kernels agree bit for bit
    assert torch.isfinite(xf).all() and torch.isfinite(xe).all()
    assert rel(bf.cpu().numpy(), be.cpu().numpy()) < REL_TOL_MEAN
    assert rel(xf.cpu().numpy(), xe.cpu().numpy()) < 1e-4


@pytest.mark.parametrize("variant", ["stream", "tile", "band"])
def test_fast_request_with_other_tv_constants_runs_exact(variant):
    """Round 6: the fast kernels are compiled for deepinv's TV constants (literal operands); a fast
    request with other constants (tau = 0.02, rho = 1.5) must run the exact kernels -- bit-identical to an exact
    request -- and the default constants keep the fast path (it differs from exact in the last bits)."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator(device=DEV).manual_seed(321)
    x = torch.rand((1, 3, 64, 64), generator=g, device=DEV)
    from psgla_for_posterior_sampling_amd.fidelity import inpainting_problem
    dg, y, init, mask2d, _ = inpainting_problem(x)
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)

    def run(exact, tau, rho):
        eng = FusedTvChains(init.expand(4, -1, -1, -1).contiguous(), y, dg.mask_u8, c1=c1, c2=c2,
                            sigma2=dg.sigma2, alpha=1.0, ths=float(np.float32(10 / 255.0)),
                            tv=K.TvConstants(tau=tau, rho=rho, n_it_max=10), seed=0, n_iter=6, n_inter=3,
                            n_inter_mmse=2, exact=exact, kernel_variant=variant)
        eng.run(6, graph_steps=0)
        torch.cuda.synchronize()
        return eng.X.clone(), eng.u2_state.clone(), eng.blocks()[0].clone()

    for a, b in zip(run(False, 0.02, 1.5), run(True, 0.02, 1.5)):
        assert torch.equal(a, b)
    xf, _, _ = run(False, 0.01, 1.99)
    xe, _, _ = run(True, 0.01, 1.99)
    assert not torch.equal(xf, xe), "default constants should take the fast kernels"
    assert _relt(xf, xe) < 1e-4


def _relt(a, b):
    return float(torch.linalg.vector_norm((a - b).double()) / torch.linalg.vector_norm(b.double()))


def test_fused_full_size_fast_vs_exact_config1_schedule():
    """The benched (fast) kernel over BASELINE configs[1]'s whole run AT ITS REAL SCHEDULE: 64 chains x
    3x256x256, N = 10000 PSGLA+TV(10) steps, n_inter = n_inter_mmse = 10 (sampling_images.py:105-106
    with N = 10000: 1,000 stored samples and 909 blocks of 11 samples), graph-replayed in 100-step
    segments, fast and exact kernels side by side on identical inputs.  The exact kernel is
    bit-identical to the CPU oracle (tests above).  Asserted against exact mode: every block mean and
    second-moment block, their means over blocks (the MMSE of sampling_images.py:428) within the
    north-star 1e-5 relative, every stored sample within 1e-4 relative.  The 64 chains run as two
    32-chain halves (chain0 = 0 / 32) so both modes' stores (71 GB each) fit in HBM together: a chain's
    values do not depend on the batch it runs in (test_fused_chains_independent_of_batching_and_graph)."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    n, half = 10000, 32
    gen = torch.Generator(device=DEV).manual_seed(0)
    mask2d = (torch.rand((256, 256), generator=gen, device=DEV) > 0.5).to(torch.uint8)
    mask = mask2d.float()[None, None]
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    worst = {"block": 0.0, "block2": 0.0, "sample": 0.0}
    for chain0 in (0, half):
        xs = torch.empty((half, 3, 256, 256), device=DEV)
        for b in range(half):
            xs[b] = torch.rand((3, 256, 256), generator=torch.Generator(device=DEV).manual_seed(1234 + chain0 + b),
                               device=DEV)
        gy = torch.Generator(device=DEV).manual_seed(100 + chain0)
        y = mask * xs + torch.normal(torch.zeros_like(xs), std=(1 / 255.0) * torch.ones_like(xs), generator=gy)
        init = (mask * y + (1 - mask) * 0.5).contiguous()
        engs = {}
        for exact in (True, False):
            eng = FusedTvChains(init, y.contiguous(), mask2d, c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)),
                                alpha=1.0, ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=10), seed=0,
                                n_iter=n, n_inter=10, n_inter_mmse=10, chain0=chain0, exact=exact)
            assert eng.main_kernel == "tv_stream_kernel"
            eng.run(n, graph_steps=100)
            engs[exact] = eng
        torch.cuda.synchronize()
        (e1, e2), (f1, f2) = engs[True].blocks(), engs[False].blocks()
        es, fs = engs[True].samples(), engs[False].samples()
        assert e1.shape[0] == 909 and f1.shape[0] == 909 and es.shape[0] == 1000 and fs.shape[0] == 1000
        assert torch.isfinite(f1).all() and torch.isfinite(fs).all()
        assert _relt(f1.mean(0), e1.mean(0)) < REL_TOL_MEAN
        assert _relt(f2.mean(0), e2.mean(0)) < REL_TOL_MEAN
        for k in range(e1.shape[0]):
            worst["block"] = max(worst["block"], _relt(f1[k], e1[k]))
            worst["block2"] = max(worst["block2"], _relt(f2[k], e2[k]))
        for k in range(es.shape[0]):
            worst["sample"] = max(worst["sample"], _relt(fs[k], es[k]))
        del engs, e1, e2, f1, f2, es, fs
        torch.cuda.empty_cache()
    print("fast vs exact, config[1] schedule, worst relative:", worst)
    assert worst["block"] < REL_TOL_MEAN and worst["block2"] < REL_TOL_MEAN
    assert worst["sample"] < 1e-4


@pytest.mark.parametrize("variant", ["stream", "tile"])
def test_fused_fast_vs_oracle_direct_10000_steps(variant):
    """Fast mode against the CPU oracle's psgla (oracle/psgla_oracle.py, the restatement of
    restoration_algorithms.py:219-271) directly, not by transitivity: 1 chain x 3x24x40, N = 10000
    steps at configs[1]'s schedule (n_inter = n_inter_mmse = 10).  Every block mean and second-moment
    block and their means over blocks within 1e-5 relative, every stored sample within 1e-4."""
    n = 10000
    eng, (dg, y, init, mask2d, c1, c2) = _fused_batch(1, 0, exact=False, n_iter=n, H=24, W=40, variant=variant,
                                                      n_inter=10, n_inter_mmse=10)
    assert eng.main_kernel == "tv_" + variant + "_kernel"
    eng.run(n, graph_steps=100)
    torch.cuda.synchronize()
    key = ("direct", n)
    if key not in _ORACLE_CACHE:
        tv = orc.TVDenoiser(n_it_max=10)
        Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(1.0), torch.tensor(10.0), sig_float=10 / 255.0,
                                delta=(10 / 255.0) ** 2, n_iter=n, n_inter=10, n_inter_mmse=10, seed=3, chain=0)
        _ORACLE_CACHE[key] = [torch.stack(v) for v in (Xl, Ml, M2l)]
    Xs, Ms, M2s = _ORACLE_CACHE[key]
    bm, bm2 = (t[:, 0].cpu() for t in eng.blocks())
    sm = eng.samples()[:, 0].cpu()
    assert bm.shape == Ms.shape and sm.shape == Xs.shape and bm.shape[0] == 909
    assert _relt(bm.mean(0), Ms.mean(0)) < REL_TOL_MEAN
    assert _relt(bm2.mean(0), M2s.mean(0)) < REL_TOL_MEAN
    wb = max(_relt(bm[k], Ms[k]) for k in range(bm.shape[0]))
    wb2 = max(_relt(bm2[k], M2s[k]) for k in range(bm.shape[0]))
    ws = max(_relt(sm[k], Xs[k]) for k in range(sm.shape[0]))
    print(f"fast {variant} vs oracle, 10000 steps, worst relative: block {wb:.3g} block2 {wb2:.3g} sample {ws:.3g}")
    assert wb < REL_TOL_MEAN and wb2 < REL_TOL_MEAN and ws < 1e-4


# ------------------------------------------------------------------------------ generic paths
def test_generic_psgla_clamp_matches_reference_fixture():
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    fx = load("psgla_inpaint_clamp")
    seed, n, ni, nm, alpha, lam, s, delta = fx["meta"]
    y = torch.from_numpy(fx["y"]).to(DEV)
    mask = torch.from_numpy(fx["mask2d"]).to(DEV)
    from psgla_for_posterior_sampling_amd.fidelity import InpaintingFidelity
    dg = InpaintingFidelity(mask, y, torch.tensor((1 / 255.0) ** 2, dtype=torch.float32))

    class Clamp:
        def forward(self, x, s):
            return torch.clamp(x, 0.0, 1.0)
    out = RA.psgla(torch.from_numpy(fx["init"]).to(DEV), dg, Clamp(), torch.tensor(alpha, dtype=torch.float32),
                   torch.tensor(lam, dtype=torch.float32), sig_float=float(s), delta=float(delta),
                   n_iter=int(n), n_inter=int(ni), n_inter_mmse=int(nm), seed=int(seed))
    Xl, Ml, M2l = [np.stack([t.cpu().numpy() for t in lst]) for lst in out]
    np.testing.assert_array_equal(Xl, fx["samples"])
    np.testing.assert_array_equal(Ml, fx["blocks"])
    np.testing.assert_array_equal(M2l, fx["blocks2"])


def test_generic_psgla_alpha03_conv_matches_reference_fixture():
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    fx = load("psgla_inpaint_conv_alpha03")
    seed, n, ni, nm, alpha, lam, s, delta = fx["meta"]
    y = torch.from_numpy(fx["y"]).to(DEV)
    mask = torch.from_numpy(fx["mask2d"]).to(DEV)
    sigma2t = torch.tensor((1 / 255.0) ** 2, dtype=torch.float32, device=DEV)
    mask4 = torch.ones(3, device=DEV)[None, :, None, None] * mask[None, None].long()
    w = torch.from_numpy(fx["weight"]).to(DEV)
    b = torch.from_numpy(fx["bias"]).to(DEV)

    class Conv:
        def forward(self, x, s):
            return x - torch.nn.functional.conv2d(x, w, b, padding=1)
    out = RA.psgla(torch.from_numpy(fx["init"]).to(DEV), lambda x: -mask4 * (x - y) / sigma2t, Conv(),
                   torch.tensor(alpha, dtype=torch.float32), torch.tensor(lam, dtype=torch.float32),
                   sig_float=float(s), delta=float(delta), n_iter=int(n), n_inter=int(ni),
                   n_inter_mmse=int(nm), seed=int(seed))
    Ml = np.stack([t.cpu().numpy() for t in out[1]])
    # the conv runs in MIOpen on the GPU vs the CPU conv in the fixture: tolerance, not bits
    assert rel(Ml.mean(0), fx["blocks"].mean(0)) < REL_TOL_MEAN


def test_generic_pnpula_clamp_matches_reference_fixture():
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.fidelity import InpaintingFidelity
    fx = load("pnpula_inpaint_clamp")
    seed, n, ni, nm, alpha, lam, s1, delta = fx["meta"]
    y = torch.from_numpy(fx["y"]).to(DEV)
    mask = torch.from_numpy(fx["mask2d"]).to(DEV)
    dg = InpaintingFidelity(mask, y, torch.tensor((1 / 255.0) ** 2, dtype=torch.float32))
    s2t = torch.tensor(float(s1) ** 2, dtype=torch.float32, device=DEV)
    alphat = torch.tensor(1.0, dtype=torch.float32, device=DEV)
    out = RA.pnpula(torch.from_numpy(fx["init"]).to(DEV), dg, lambda x: alphat * (torch.clamp(x, 0, 1) - x) / s2t,
                    torch.tensor(float(delta), dtype=torch.float32, device=DEV),
                    torch.tensor(float(lam), dtype=torch.float32, device=DEV), n_iter=int(n), n_inter=int(ni),
                    n_inter_mmse=int(nm), seed=int(seed))
    Xl, Ml, M2l = [np.stack([t.cpu().numpy() for t in lst]) for lst in out]
    np.testing.assert_array_equal(Xl, fx["samples"])
    np.testing.assert_array_equal(Ml, fx["blocks"])
    np.testing.assert_array_equal(M2l, fx["blocks2"])


def test_inpaint_grad_bitwise():
    from psgla_for_posterior_sampling_amd.fidelity import InpaintingFidelity
    fx = load("psgla_inpaint_clamp")
    dg_ref, y, init, mask2d = orc.inpainting_problem(torch.from_numpy(fx["x"]), seed_ip=0)
    dg = InpaintingFidelity(mask2d.to(DEV), y.to(DEV), torch.tensor((1 / 255.0) ** 2, dtype=torch.float32))
    x = torch.rand(init.shape)
    np.testing.assert_array_equal(dg(x.to(DEV)).cpu().numpy(), dg_ref(x).numpy())


# ---------------------------------------------------------------------------------------
# Deblurring data term (HIP stencil) -- sampling_images.py:304-341
# ---------------------------------------------------------------------------------------
def _blur_case(B, H, W, l, bt, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((B, 3, H, W), generator=g)
    A, AT = orc.blur_operators(l=l, blur_type=bt)
    y = A(x) + torch.normal(torch.zeros_like(x), (1 / 255.0) * torch.ones_like(x), generator=g)
    xs = (x + 0.05 * torch.randn(x.shape, generator=g)).contiguous()
    s2 = torch.tensor((1 / 255.0) ** 2, dtype=torch.float32)
    ref = -AT(A(xs) - y) / s2           # the reference's closure, torch CPU
    return xs, y, ref


# the stencil sums 2 x 81 products in its own order (torch's CPU conv2d order is not specified),
# so parity is a tolerance: |g - g_ref| <= BLUR_TOL * max|g_ref|; A x - y cancels to the noise
# level, which amplifies fp32 rounding of the 81-term sums by ~100x relative to |g|.
BLUR_TOL = 2e-5


@pytest.mark.parametrize("B,H,W,l,bt", [(2, 40, 52, 4, "uniform"), (1, 37, 29, 4, "gaussian"),
                                        (2, 70, 130, 2, "uniform"), (1, 16, 16, 0, "uniform"),
                                        (1, 45, 71, 3, "gaussian"), (1, 130, 200, 5, "uniform")])
@pytest.mark.parametrize("exact", [True, False])
def test_blur_grad_matches_reference_closure(B, H, W, l, bt, exact):
    from psgla_for_posterior_sampling_amd import hip_ops as K
    xs, y, ref = _blur_case(B, H, W, l, bt, seed=B * H + W)
    h_ = orc.blur_kernel(l, bt)
    hconv = torch.from_numpy(np.copy(np.flip(h_))).float().to(DEV)
    hcorr = torch.from_numpy(h_).float().to(DEV)
    g = K.blur_grad(xs.to(DEV), y.to(DEV), hconv, hcorr, l, float(np.float32((1 / 255.0) ** 2)), exact=exact)
    torch.cuda.synchronize()
    err = (g.cpu() - ref).abs().max().item()
    assert err <= BLUR_TOL * ref.abs().max().item(), err


@pytest.mark.parametrize("B,H,W,l", [(2, 40, 52, 4), (1, 37, 29, 4), (2, 70, 130, 2), (1, 16, 16, 0),
                                     (1, 45, 70, 3), (1, 50, 44, 8), (1, 130, 200, 4), (1, 33, 40, 6)])
def test_blur_grad_exact_bitwise_vs_tap_order_oracle(B, H, W, l):
    """Exact mode sums every output's (2l+1)^2 products in (row, column) tap order with IEEE
    multiply / add / divide: bit-identical to oracle.blur_grad_tap_order on odd widths, partial
    tiles, several tiles per plane, odd and even l (LDS-DMA and register staging)."""
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator().manual_seed(H * W + l)
    x = torch.rand((B, 3, H, W), generator=g)
    y = torch.rand((B, 3, H, W), generator=g)
    h_ = orc.blur_kernel(l, "gaussian").astype(np.float32)
    hconv = np.flip(h_).copy()
    s2 = float(np.float32((1 / 255.0) ** 2))
    got = K.blur_grad(x.to(DEV), y.to(DEV), torch.from_numpy(hconv), torch.from_numpy(h_), l, s2, exact=True)
    torch.cuda.synchronize()
    want = orc.blur_grad_tap_order(x.numpy(), y.numpy(), hconv, h_, l, s2)
    np.testing.assert_array_equal(got.cpu().numpy(), want)


def test_blur_fast_separable_path():
    """Fast mode runs the reference's rank-1 (h^T h) taps as separable row / column passes: within fp32
    rounding of the 2-D stencil (3e-6 of max|g| measured on a real deblurring observation, where A x - y
    cancels; bound 1e-5, half the 2e-5 contract against the reference closure, which it also meets);
    taps that are not rank 1 stay on the 2-D stencil (bitwise equal to it)."""
    from psgla_for_posterior_sampling_amd import hip_ops as K
    xs, y, ref = _blur_case(2, 70, 130, 4, "gaussian", seed=11)
    h_ = orc.blur_kernel(4, "gaussian")
    hconv = torch.from_numpy(np.copy(np.flip(h_))).float()
    hcorr = torch.from_numpy(h_).float()
    s2 = float(np.float32((1 / 255.0) ** 2))
    X, yd = xs.to(DEV), y.to(DEV)
    try:
        g_sep = K.blur_grad(X, yd, hconv, hcorr, 4, s2).cpu()
        K.blur_set_separable(False)
        g_2d = K.blur_grad(X, yd, hconv, hcorr, 4, s2).cpu()
        assert (g_sep - g_2d).abs().max().item() <= 1e-5 * g_2d.abs().max().item()
        assert (g_sep - ref).abs().max().item() <= BLUR_TOL * ref.abs().max().item()
        # a full-rank tap set: the 2-D stencil either way
        hr = torch.rand((9, 9), generator=torch.Generator().manual_seed(3))
        hr = hr / hr.sum()
        g_a = K.blur_grad(X, yd, hr, hr.t().contiguous(), 4, s2).cpu()
        K.blur_set_separable(True)
        g_b = K.blur_grad(X, yd, hr, hr.t().contiguous(), 4, s2).cpu()
        torch.cuda.synchronize()
        assert torch.equal(g_a, g_b)
    finally:
        K.blur_set_separable(True)


def test_blur_langevin_fused_equals_grad_then_update():
    """The fused stencil + Langevin kernel == blur_grad followed by langevin_update (same noise)."""
    from psgla_for_posterior_sampling_amd import hip_ops as K
    xs, y, _ = _blur_case(2, 40, 52, 4, "uniform", seed=3)
    h_ = orc.blur_kernel(4, "uniform")
    hconv = torch.from_numpy(np.copy(np.flip(h_))).float().to(DEV)
    hcorr = torch.from_numpy(h_).float().to(DEV)
    X, yd = xs.to(DEV), y.to(DEV)
    s2 = float(np.float32((1 / 255.0) ** 2))
    for W in (52, 30):                                  # quad-aligned and per-element noise paths
        Xw, yw = X[..., :W].contiguous(), yd[..., :W].contiguous()
        g = K.blur_grad(Xw, yw, hconv, hcorr, 4, s2, exact=True)
        Y1 = K.langevin_update(Xw, g, 1e-4, 0.05, seed=9, chain0=3, step=17)
        Y2 = K.blur_langevin(Xw, yw, hconv, hcorr, 4, s2, 1e-4, 0.05, seed=9, chain0=3, step=17, exact=True)
        torch.cuda.synchronize()
        assert torch.equal(Y1, Y2)


@pytest.mark.parametrize("bt", ["uniform", "gaussian"])
def test_generic_psgla_deblur_matches_reference_fixture(bt):
    """psgla with the HIP deblurring step (fused stencil + Langevin) vs the reference's own run
    (tests/golden psgla_deblur_*: clamp denoiser, 60 steps): sample means within REL_TOL_MEAN."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.fidelity import BlurFidelity
    fx = load(f"psgla_deblur_{bt}")
    seed, n, ni, nm, alpha, lam, s, delta, l = fx["meta"]
    l = int(l)
    hcorr = torch.from_numpy(fx["hcorr"]).float()
    hconv = torch.flip(hcorr, dims=(0, 1)).contiguous()
    ones = torch.ones(3, 2 * l + 1, 2 * l + 1)
    dg = BlurFidelity((hconv[None, None] * ones[:, None]).to(DEV), (hcorr[None, None] * ones[:, None]).to(DEV), l,
                      torch.from_numpy(fx["y"]).to(DEV), torch.tensor((1 / 255.0) ** 2, dtype=torch.float32))

    class Clamp:
        def forward(self, x, s):
            return torch.clamp(x, 0.0, 1.0)
    out = RA.psgla(torch.from_numpy(fx["init"]).to(DEV), dg, Clamp(), torch.tensor(alpha, dtype=torch.float32),
                   torch.tensor(lam, dtype=torch.float32), sig_float=float(s), delta=float(delta),
                   n_iter=int(n), n_inter=int(ni), n_inter_mmse=int(nm), seed=int(seed))
    Xl, Ml, M2l = [np.stack([t.cpu().numpy() for t in lst]) for lst in out]
    assert Xl.shape == fx["samples"].shape and Ml.shape == fx["blocks"].shape
    assert rel(Ml.mean(0), fx["blocks"].mean(0)) < REL_TOL_MEAN
    assert rel(M2l.mean(0), fx["blocks2"].mean(0)) < REL_TOL_MEAN


@pytest.mark.parametrize("B,H,W,alpha", [(2, 23, 29, 1.0), (2, 19, 31, 1.0), (2, 21, 33, 0.6), (2, 16, 61, 1.0),
                                         (2, 13, 301, 1.0), (2, 11, 483, 1.0),
                                         # half-wave windows (256 < W <= 324): 3 segments of <= 128 columns, two per
                                         # wave; B = 1: 9 segments, the last pair's second half disabled
                                         (1, 17, 321, 1.0), (2, 15, 290, 0.6)])
def test_stream_padded_rows_exact_vs_oracle(B, H, W, alpha):
    """W % 4 != 0 (rows padded to a multiple of 4 columns, the lane's 4 noise elements spanning two
    quads at every offset) and W > 256 (column segments; for 256 < W <= 324 half-wave windows, a pair of
    segments per wave): the streaming kernel, bit-identical."""
    eng, (dg, y, init, mask2d, c1, c2) = _fused_batch(B, 5, exact=True, n_iter=12, H=H, W=W, alpha=alpha,
                                                      variant="stream")
    assert eng.main_kernel == "tv_stream_kernel"
    eng.run(12, graph_steps=0)
    torch.cuda.synchronize()
    bm, bm2 = eng.blocks()
    for b in range(B):
        tv = orc.TVDenoiser(n_it_max=10)
        Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(alpha), torch.tensor(10.0), sig_float=10 / 255.0,
                                delta=(10 / 255.0) ** 2, n_iter=12, n_inter=5, n_inter_mmse=4, seed=3, chain=5 + b)
        np.testing.assert_array_equal(eng.samples()[:, b].cpu().numpy(), np.stack([t.numpy() for t in Xl]))
        np.testing.assert_array_equal(bm[:, b].cpu().numpy(), np.stack([t.numpy() for t in Ml]))
        np.testing.assert_array_equal(bm2[:, b].cpu().numpy(), np.stack([t.numpy() for t in M2l]))
        np.testing.assert_array_equal(eng.u2_state[b].cpu().numpy(), tv.u2.numpy()[0])
        np.testing.assert_array_equal(eng.x2_state[b].cpu().numpy(), tv.x2.numpy()[0])


def test_psgla_padded_rows_returns_reference_shapes():
    """The drop-in psgla() on an odd-width image: lists of (C, H, W) tensors, warm TV state (C, H, W)."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.denoisers import TVDenoiser
    from psgla_for_posterior_sampling_amd.fidelity import InpaintingFidelity
    g = torch.Generator().manual_seed(2)
    x = torch.rand((1, 3, 21, 37), generator=g)
    dg_ref, y, init, mask2d = orc.inpainting_problem(x, seed_ip=0)
    dg = InpaintingFidelity(mask2d.to(DEV), y.to(DEV), torch.tensor((1 / 255.0) ** 2, dtype=torch.float32))
    den = TVDenoiser(n_it_max=10, exact=True)
    s = 10 / 255.0
    out = RA.psgla(init.to(DEV), dg, den, torch.tensor(1.0), torch.tensor(10.0), sig_float=s, delta=s ** 2,
                   n_iter=20, n_inter=10, n_inter_mmse=9, seed=0)
    ref = orc.psgla(init, dg_ref, orc.TVDenoiser(n_it_max=10), torch.tensor(1.0), torch.tensor(10.0), sig_float=s,
                    delta=s ** 2, n_iter=20, n_inter=10, n_inter_mmse=9, seed=0)
    for a, b in zip(out, ref):
        assert len(a) == len(b) > 0
        for u, v in zip(a, b):
            assert tuple(u.shape) == (3, 21, 37)
            np.testing.assert_array_equal(u.cpu().numpy(), v.numpy())
    assert tuple(den.x2.shape) == (1, 3, 21, 37) and den.x2.is_contiguous()
    assert tuple(den.u2.shape) == (1, 3, 21, 37, 2)


@pytest.mark.parametrize("W,stream_wgs", [(301, 0), (301, 4), (301, 7), (301, 33), (483, 0), (483, 9), (300, 6)])
def test_stream_segmented_row_split_exact_vs_oracle(W, stream_wgs):
    """W > 256: rows of every (plane, column segment) pair cut into ranges over the CUs (ranges
    crossing segment and plane boundaries, n_tv halo rows at cuts): bit-identical to the checker."""
    B, H, n_iter = 2, 20, 10
    eng, (dg, y, init, mask2d, c1, c2) = _fused_batch(B, 7, exact=True, n_iter=n_iter, H=H, W=W,
                                                      variant="stream", stream_wgs=stream_wgs)
    eng.run(n_iter, graph_steps=0)
    torch.cuda.synchronize()
    bm, bm2 = eng.blocks()
    for b in range(B):
        tv = orc.TVDenoiser(n_it_max=10)
        Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(1.0), torch.tensor(10.0), sig_float=10 / 255.0,
                                delta=(10 / 255.0) ** 2, n_iter=n_iter, n_inter=5, n_inter_mmse=4, seed=3,
                                chain=7 + b)
        np.testing.assert_array_equal(eng.samples()[:, b].cpu().numpy(), np.stack([t.numpy() for t in Xl]))
        np.testing.assert_array_equal(bm[:, b].cpu().numpy(), np.stack([t.numpy() for t in Ml]))
        np.testing.assert_array_equal(eng.u2_state[b].cpu().numpy(), tv.u2.numpy()[0])


def test_stream_segmented_early_stop_exact_vs_oracle():
    """Early stop with padded rows and column segments: the last workgroup re-streams every
    (plane, segment) of the stopped chains -- bit-identical."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    B, H, W, n_iter, tol = 2, 18, 263, 10, 3e-2
    g = torch.Generator().manual_seed(9)
    x = torch.rand((1, 3, H, W), generator=g)
    dg, y, init, mask2d = orc.inpainting_problem(x, seed_ip=3)
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    eng = FusedTvChains(init.expand(B, -1, -1, -1).contiguous().to(DEV), y.to(DEV), mask2d.to(torch.uint8).to(DEV),
                        c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)), alpha=1.0,
                        ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=10, tol=tol), seed=4,
                        n_iter=n_iter, n_inter=3, n_inter_mmse=2, exact=True, kernel_variant="stream")
    eng.run(n_iter, graph_steps=0)
    torch.cuda.synchronize()
    fired = False
    for b in range(B):
        tv = _RecordingTV(n_it_max=10, tol=tol)
        Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(1.0), torch.tensor(10.0), sig_float=10 / 255.0,
                                delta=(10 / 255.0) ** 2, n_iter=n_iter, n_inter=3, n_inter_mmse=2, seed=4, chain=b)
        fired = fired or min(tv.its) < 10
        np.testing.assert_array_equal(eng.samples()[:, b].cpu().numpy(), np.stack([t.numpy() for t in Xl]))
        np.testing.assert_array_equal(eng.u2_state[b].cpu().numpy(), tv.u2.numpy()[0])
    assert fired, "test needs the early stop to fire"


@pytest.mark.parametrize("variant", ["stream", "tile", "band"])
def test_fused_single_channel_exact_vs_oracle(variant):
    """One-channel (grayscale, --grayscale) images: the fused step with C = 1 is bit-identical to the oracle
    on the same data term (-mask * (x - y) / sigma2, sampling_images.py:295 with a one-channel mask)."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    H, W, B, n_iter = 40, 52, 2, 12
    g = torch.Generator().manual_seed(11)
    x = torch.rand((1, 1, H, W), generator=g)
    gm = torch.Generator().manual_seed(3)
    mask_2d = 1 * (torch.rand((H, W), generator=gm) > 0.5)
    mask = torch.ones(1)[None, :, None, None] * mask_2d[None, None, :, :]
    sigma1 = 1 / 255.0
    sigma2t = torch.tensor(sigma1 ** 2, dtype=torch.float32)
    y = mask * x + torch.normal(torch.zeros(*x.size()), std=sigma1 * torch.ones(*x.size()), generator=gm)
    init = mask * y + (1 - mask) * 0.5 * torch.ones(y.shape)

    def dg(v):
        return -mask * (v - y) / sigma2t
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    eng = FusedTvChains(init.expand(B, -1, -1, -1).contiguous().to(DEV), y.to(DEV), mask_2d.to(torch.uint8).to(DEV),
                        c1=c1, c2=c2, sigma2=float(np.float32(sigma1 ** 2)), alpha=1.0, ths=float(np.float32(10 / 255.0)),
                        tv=K.TvConstants(n_it_max=10), seed=7, n_iter=n_iter, n_inter=3, n_inter_mmse=2, exact=True,
                        kernel_variant=variant)
    assert eng.main_kernel == {"stream": "tv_stream_kernel", "tile": "tv_tile_kernel", "band": "tv_main_kernel"}[variant]
    eng.run(n_iter, graph_steps=0)
    torch.cuda.synchronize()
    bm, bm2 = eng.blocks()
    for b in range(B):
        tv = orc.TVDenoiser(n_it_max=10)
        Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(1.0), torch.tensor(10.0), sig_float=10 / 255.0,
                                delta=(10 / 255.0) ** 2, n_iter=n_iter, n_inter=3, n_inter_mmse=2, seed=7, chain=b)
        # the oracle's lists hold squeezed tensors (restoration_algorithms.py:244: torch.squeeze drops C = 1)
        np.testing.assert_array_equal(eng.samples()[:, b, 0].cpu().numpy(), np.stack([t.numpy() for t in Xl]))
        np.testing.assert_array_equal(bm[:, b, 0].cpu().numpy(), np.stack([t.numpy() for t in Ml]))
        np.testing.assert_array_equal(bm2[:, b, 0].cpu().numpy(), np.stack([t.numpy() for t in M2l]))


def test_auto_dispatch_by_shape():
    """64 chains x 3 x 256 x 256 (BASELINE configs[1], one GPU): auto dispatch picks the row stream; 8 chains
    (the 8-GPU strong split) and 16 (the 4-GPU split) the tile kernel; alpha != 1 and many chains of a real shape the row stream; one
    or two chains of a real shape (padded rows, column segments) the tile kernel."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K

    def kern(B, H, W, alpha=1.0):
        z = torch.zeros((B, 3, H, W), device=DEV)
        return FusedTvChains(z, z[:1].clone(), torch.ones((H, W), dtype=torch.uint8, device=DEV), c1=0.1, c2=0.1,
                             sigma2=1e-5, alpha=alpha, ths=0.04, tv=K.TvConstants(n_it_max=10), seed=0, n_iter=10,
                             n_inter=10, n_inter_mmse=10, store_samples=False, store_blocks=False).main_kernel
    assert kern(64, 256, 256) == "tv_stream_kernel"
    assert kern(8, 256, 256) == "tv_tile_kernel"
    assert kern(64, 256, 256, alpha=0.6) == "tv_stream_kernel"
    assert kern(16, 321, 481) == "tv_stream_kernel"
    assert kern(1, 481, 321) == "tv_tile_kernel"        # castle at the CLI's B = 1: 3 x 2 x 19 tiles
    assert kern(2, 321, 481) == "tv_tile_kernel"
    assert kern(4, 481, 321) == "tv_tile_kernel"        # two rounds of tiles beat segmented row streams
    assert kern(8, 481, 321) == "tv_stream_kernel"
    # since round 6 no 72-row tiles (they spilled VGPRs): 12-16 chains run 48-row tiles in two rounds
    assert kern(12, 256, 256) == "tv_tile_kernel"
    assert kern(16, 256, 256) == "tv_tile_kernel"       # the 4-GPU strong split: 480 tiles
    assert kern(20, 256, 256) == "tv_stream_kernel"     # 600 tiles: three rounds
    assert kern(8, 256, 256, alpha=0.6) == "tv_stream_kernel"   # 48-row tiles only at alpha = 1


# ------------------------------------------------------------------------------ small-batch tile kernel
@pytest.mark.parametrize("B,H,W,alpha,tol,n_tv", [(3, 48, 64, 1.0, 1e-5, 10), (2, 100, 64, 1.0, 1e-5, 10),
                                                  (2, 77, 40, 0.6, 1e-5, 10), (2, 40, 52, 1.0, 3e-2, 10),
                                                  (2, 90, 256, 1.0, 1e-5, 3), (1, 30, 20, 1.0, 1e-5, 14),
                                                  # padded rows / column segments (GEN tiles)
                                                  (2, 37, 29, 1.0, 1e-5, 10), (1, 60, 300, 1.0, 1e-5, 10),
                                                  (1, 33, 483, 0.6, 1e-5, 10), (2, 70, 301, 1.0, 3e-2, 10),
                                                  (1, 50, 257, 1.0, 1e-5, 4), (1, 3, 321, 1.0, 1e-5, 10),
                                                  # enough tiles that 32-row tiles would need two rounds:
                                                  # 48-row tiles (3 rows per wave), plain and segmented
                                                  (12, 100, 64, 1.0, 1e-5, 10), (24, 40, 301, 1.0, 3e-2, 10),
                                                  # more than one round of 48-row tiles: two rounds (the
                                                  # serial early-stop recompute; no 72-row tiles since round 6)
                                                  (24, 100, 64, 1.0, 1e-5, 10), (24, 130, 64, 1.0, 3e-2, 10),
                                                  # one- and two-row images, one inner iteration
                                                  (2, 1, 40, 1.0, 1e-5, 10), (1, 2, 321, 1.0, 1e-5, 10),
                                                  (2, 37, 64, 1.0, 1e-5, 1)])
def test_tile_kernel_exact_vs_oracle(B, H, W, alpha, tol, n_tv):
    """The small-batch tile kernel (one 32- or 48-row tile per workgroup, n_tv halo rows at band cuts,
    inline finalisation) in exact mode: samples, block means and TV state bit-identical to the CPU oracle
    for band cuts, narrow images (idle lanes), alpha != 1, deepinv's early stop and n_tv > 10; for rows
    padded to a pitch (W % 4 != 0) and column segments with n_tv halo columns (W > 256); 32-row tiles
    where they fit on the CUs in one round, 48-row tiles for the larger batches, in two rounds where they
    do not fit in one (the serial early-stop recompute)."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator().manual_seed(9)
    x = torch.rand((1, 3, H, W), generator=g)
    dg, y, init, mask2d = orc.inpainting_problem(x, seed_ip=2)
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    n_iter = 14
    eng = FusedTvChains(init.expand(B, -1, -1, -1).contiguous().to(DEV), y.to(DEV), mask2d.to(torch.uint8).to(DEV),
                        c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)), alpha=alpha,
                        ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=n_tv, tol=tol), seed=6,
                        n_iter=n_iter, n_inter=3, n_inter_mmse=2, chain0=4, exact=True, kernel_variant="tile")
    assert eng.main_kernel == "tv_tile_kernel"
    eng.run(n_iter, graph_steps=6)
    torch.cuda.synchronize()
    bm, bm2 = eng.blocks()
    for b in range(B):
        tv = orc.TVDenoiser(n_it_max=n_tv, tol=tol)
        Xl, Ml, M2l = orc.psgla(init, dg, tv, torch.tensor(alpha), torch.tensor(10.0), sig_float=10 / 255.0,
                                delta=(10 / 255.0) ** 2, n_iter=n_iter, n_inter=3, n_inter_mmse=2, seed=6, chain=4 + b)
        # (the oracle's lists hold squeezed tensors: a one-row image loses its H axis there)
        sm = eng.samples()[:, b].cpu().numpy()
        np.testing.assert_array_equal(sm, np.stack([t.numpy() for t in Xl]).reshape(sm.shape))
        np.testing.assert_array_equal(bm[:, b].cpu().numpy(), np.stack([t.numpy() for t in Ml]).reshape(bm[:, b].shape))
        np.testing.assert_array_equal(bm2[:, b].cpu().numpy(), np.stack([t.numpy() for t in M2l]).reshape(bm2[:, b].shape))
        np.testing.assert_array_equal(eng.x2_state[b].cpu().numpy(), tv.x2.numpy()[0])
        np.testing.assert_array_equal(eng.u2_state[b].cpu().numpy(), tv.u2.numpy()[0])


@pytest.mark.parametrize("B", [8, 16])
def test_tile_kernel_equals_stream_kernel_full_size(B):
    """Strong-scaling batch sizes at the benched image size (3 x 256 x 256): the tile kernel and the
    row-streaming kernel give bit-identical chains in both arithmetic modes (the same per-element
    operations; the exact stream kernel is bit-identical to the oracle)."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator(device=DEV).manual_seed(1234)
    xs = torch.rand((B, 3, 256, 256), generator=g, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(0)
    mask2d = (torch.rand((256, 256), generator=gen, device=DEV) > 0.5).to(torch.uint8)
    y = mask2d.float() * xs + torch.normal(torch.zeros_like(xs), std=(1 / 255.0) * torch.ones_like(xs),
                                           generator=gen)
    init = (mask2d.float() * y + (1 - mask2d.float()) * 0.5).contiguous()
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    for exact in (True, False):
        outs = []
        for variant in ("stream", "tile"):
            eng = FusedTvChains(init, y.contiguous(), mask2d, c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)),
                                alpha=1.0, ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=10), seed=0,
                                n_iter=30, n_inter=10, n_inter_mmse=10, exact=exact, kernel_variant=variant)
            eng.run(30, graph_steps=10)
            torch.cuda.synchronize()
            bm, bm2 = eng.blocks()
            outs.append((eng.samples().clone(), bm.clone(), bm2.clone(), eng.X.clone(), eng.u2_state.clone()))
        for a, b in zip(*outs):
            assert torch.equal(a, b), f"exact={exact}"


@pytest.mark.parametrize("B,H,W", [(1, 481, 321), (2, 321, 481), (1, 100, 522)])
def test_tile_kernel_equals_stream_kernel_real_shapes(B, H, W):
    """The reference's image shapes (set1c castle 481 x 321, CBSD68 321 x 481) at the CLI's batch sizes:
    the tile kernel with padded rows and column segments gives chains bit-identical to the row-streaming
    kernel (same segment geometry, same per-element operations), in both arithmetic modes."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator(device=DEV).manual_seed(77)
    xs = torch.rand((B, 3, H, W), generator=g, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(0)
    mask2d = (torch.rand((H, W), generator=gen, device=DEV) > 0.5).to(torch.uint8)
    y = mask2d.float() * xs + torch.normal(torch.zeros_like(xs), std=(1 / 255.0) * torch.ones_like(xs),
                                           generator=gen)
    init = (mask2d.float() * y + (1 - mask2d.float()) * 0.5).contiguous()
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    for exact in (True, False):
        outs = []
        for variant in ("stream", "tile"):
            eng = FusedTvChains(init, y.contiguous(), mask2d, c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)),
                                alpha=1.0, ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=10), seed=0,
                                n_iter=24, n_inter=5, n_inter_mmse=4, exact=exact, kernel_variant=variant)
            assert eng.main_kernel == "tv_" + variant + "_kernel"
            eng.run(24, graph_steps=8)
            torch.cuda.synchronize()
            bm, bm2 = eng.blocks()
            outs.append((eng.samples().clone(), bm.clone(), bm2.clone(), eng.X.clone(), eng.u2_state.clone()))
        for a, b in zip(*outs):
            assert torch.equal(a, b), f"exact={exact}"


@pytest.mark.parametrize("B,H,W,tol", [(8, 256, 256, 3e-3), (8, 256, 256, 1e-3), (16, 256, 256, 3e-3),
                                       (1, 481, 321, 3e-3), (2, 321, 481, 3e-3), (1, 256, 256, 3e-3),
                                       (2, 256, 256, 3e-3)])
def test_tile_kernel_early_stop_handoff_full_size(B, H, W, tol):
    """The tile kernel's fence-free step hand-off (sc1 stores, rel-err sums as agent atomics read back by
    the last workgroup's agent atomics) under a tolerance at which deepinv's early stop fires: 40 steps of
    8 chains (48-row tiles) or 16 chains (48-row tiles in two rounds: the serial recompute) at 3 x 256 x 256, the reference's real shapes at
    the CLI's batch sizes (castle 481 x 321 at B = 1, 321 x 481 at B = 2) and 256 x 256 at B = 1, 2 (32-row
    tiles): >= 64 tiles per chain, so the rel-err sums are spread over the workspace's 8 norm copies (ABI 8;
    read back to back and reset by exchange since round 4), bit-identical to the row-streaming
    kernel (which keeps its release / acquire fences and one norm copy), and different from the same run
    without early stops (so stops did fire).  After every run the whole norms workspace (all copies) is
    zero again: the finaliser summed and cleared every copy."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator(device=DEV).manual_seed(77)
    xs = torch.rand((B, 3, H, W), generator=g, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(0)
    mask2d = (torch.rand((H, W), generator=gen, device=DEV) > 0.5).to(torch.uint8)
    y = mask2d.float() * xs + torch.normal(torch.zeros_like(xs), std=(1 / 255.0) * torch.ones_like(xs),
                                           generator=gen)
    init = (mask2d.float() * y + (1 - mask2d.float()) * 0.5).contiguous()
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    outs = {}
    for variant, t in (("stream", tol), ("tile", tol), ("tile", 1e-5)):
        eng = FusedTvChains(init, y.contiguous(), mask2d, c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)),
                            alpha=1.0, ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=10, tol=t),
                            seed=0, n_iter=40, n_inter=10, n_inter_mmse=10, kernel_variant=variant)
        assert eng.main_kernel == "tv_" + variant + "_kernel"
        eng.run(40, graph_steps=10)
        torch.cuda.synchronize()
        assert eng.work.copies == 8
        assert not torch.any(eng.work.norms_all != 0).item(), "norm copies left non-zero after a step"
        assert int(eng.work.arrive[0].item()) == 0, "arrival counter not reset"
        eng.check_handoff()
        bm, bm2 = eng.blocks()
        outs[(variant, t)] = (eng.samples().clone(), bm.clone(), bm2.clone(), eng.X.clone(), eng.u2_state.clone())
    for a, b in zip(outs[("stream", tol)], outs[("tile", tol)]):
        assert torch.equal(a, b)
    assert not torch.equal(outs[("tile", tol)][3], outs[("tile", 1e-5)][3]), "no early stop fired"


@pytest.mark.parametrize("B,H,W,variant,stream_wgs", [(64, 256, 256, "stream", 0), (64, 481, 321, "stream", 0),
                                                       (6, 40, 52, "stream", -1), (8, 256, 256, "tile", 0),
                                                       (1, 481, 321, "tile", 0), (24, 130, 64, "tile", 0)])
def test_parallel_early_stop_redo_equals_serial(B, H, W, variant, stream_wgs):
    """ABI 11: when deepinv's early stop fires in the row stream or the tile kernel, the next launch's workgroups
    redo the stopped chains' part of the step in parallel (each its own rows / tile, then a grid barrier), the
    run's last step through launch_mask 4; the finaliser's serial recompute (no redo buffer) is the reference.
    tol = 0.2 makes the stop fire on every
    chain in every step (after 3 inner iterations), tol = 2e-3 on some steps only; fast kernels, hipGraph replay,
    the bench shape (64 chains: row split, 256 workgroups), the castle shape at 64 chains (half-wave windows,
    segments), per-plane streams, the 8-chain tile kernel, castle at batch 1 and 48-row tiles in two rounds (the
    serial recompute in both legs): bit-identical."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator(device=DEV).manual_seed(5)
    xs = torch.rand((B, 3, H, W), generator=g, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(0)
    mask2d = (torch.rand((H, W), generator=gen, device=DEV) > 0.5).to(torch.uint8)
    y = mask2d.float() * xs
    init = (mask2d.float() * y + (1 - mask2d.float()) * 0.5).contiguous()
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    for tol in (0.2, 2e-3):
        outs = []
        for par in (True, False):
            eng = FusedTvChains(init, y.contiguous(), mask2d, c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)),
                                alpha=1.0, ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=10, tol=tol),
                                seed=1, n_iter=24, n_inter=3, n_inter_mmse=4, kernel_variant=variant,
                                stream_wgs=stream_wgs, parallel_redo=par)
            assert eng.main_kernel == "tv_" + variant + "_kernel"
            eng.run(5)                         # eager steps: each launch redoes the previous step's stops
            eng.run(19, graph_steps=6)         # graph replays, then eager remainder + settle
            torch.cuda.synchronize()
            eng.check_handoff()
            assert int(eng.work.redo[0].item()) == 0 and int(eng.work.arrive[0].item()) == 0
            bm, bm2 = eng.blocks()
            outs.append((eng.samples().clone(), bm.clone(), bm2.clone(), eng.X.clone(), eng.u2_state.clone()))
        for a, b in zip(*outs):
            assert torch.equal(a, b), (tol, B, H, W, variant)


@pytest.mark.parametrize("variant,B,H,W,stream_wgs", [("stream", 6, 40, 52, -1), ("tile", 2, 100, 64, 0),
                                                      ("tile", 1, 61, 301, 0)])
@pytest.mark.parametrize("exact,alpha,warm", [(True, 1.0, False), (False, 0.6, False), (True, 0.6, False),
                                              (False, 1.0, True), (False, 0.6, True)])
def test_parallel_early_stop_redo_modes(variant, B, H, W, stream_wgs, exact, alpha, warm):
    """The parallel early-stop redo (ABI 11) on the paths the fast alpha = 1 cold-start cases above do not take
    (ADVICE r5): exact arithmetic, the alpha != 1 TV primal ping-pong (x2) the redo must read from the stopped
    step's parity, and a warm start from a previous run's (x2, u2), whose first step runs with its own descriptor
    (step() settles it with that descriptor).  tol = 0.2: the stop fires on every chain in every step.
    Parallel == serial recompute, bit for bit; input_state() of the last step is settled."""
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator(device=DEV).manual_seed(15)
    xs = torch.rand((B, 3, H, W), generator=g, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(3)
    mask2d = (torch.rand((H, W), generator=gen, device=DEV) > 0.5).to(torch.uint8)
    y = mask2d.float() * xs
    init = (mask2d.float() * y + (1 - mask2d.float()) * 0.5).contiguous()
    tv_x2 = tv_u2 = None
    if warm:
        tv_x2 = (init + 0.01 * torch.rand(init.shape, generator=g, device=DEV)).contiguous()
        tv_u2 = (0.02 * torch.rand(init.shape + (2,), generator=g, device=DEV) - 0.01).contiguous()
    c1, c2 = orc.psgla_coefficients((10 / 255.0) ** 2, 10.0, 10 / 255.0)
    outs = []
    for par in (True, False):
        eng = FusedTvChains(init, y.contiguous(), mask2d, c1=c1, c2=c2, sigma2=float(np.float32((1 / 255.0) ** 2)),
                            alpha=alpha, ths=float(np.float32(10 / 255.0)), tv=K.TvConstants(n_it_max=10, tol=0.2),
                            seed=2, n_iter=16, n_inter=3, n_inter_mmse=4, kernel_variant=variant, exact=exact,
                            stream_wgs=stream_wgs, parallel_redo=par, tv_x2=tv_x2, tv_u2=tv_u2)
        assert eng.main_kernel == "tv_" + variant + "_kernel"
        eng.run(4)
        last_in = eng.input_state(eng.steps_done).clone()     # settles the pending redo of step 3
        eng.run(12, graph_steps=4)
        torch.cuda.synchronize()
        eng.check_handoff()
        assert int(eng.work.redo[0].item()) == 0 and int(eng.work.arrive[0].item()) == 0
        bm, bm2 = eng.blocks()
        outs.append((last_in, eng.samples().clone(), bm.clone(), bm2.clone(), eng.X.clone(), eng.u2_state.clone(),
                     eng.x2_state.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b), (variant, exact, alpha, warm)
