"""GPU tests of the DNN-denoiser paths (BASELINE configs 3-5): the fused epilogue/prologue pass
(psgla_relax_langevin_inpaint), the hipGraph-replayed engines DenoiserChains / UlaChains against
the step-by-step generic loop (same kernels, same denoiser: bit for bit), and against the CPU
oracle (restoration_algorithms.py restated) within the north-star tolerance -- the convolutions
run in MIOpen on the GPU and in ATen on the CPU, so the denoiser itself is not bit-identical."""
import os

import numpy as np
import pytest
import torch

from oracle import psgla_oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
REL_TOL_MEAN = 1e-5   # north-star tolerance on the sample mean (fp32)


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


def small_dncnn(seed=0, depth=5):
    from psgla_for_posterior_sampling_amd.denoisers import DnCNN
    torch.manual_seed(seed)
    m = DnCNN(depth=depth, nf=16)
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(0.3)
    return m


def problem(B=2, H=32, W=48, deblur=False, seed=1):
    from psgla_for_posterior_sampling_amd.fidelity import deblurring_problem, inpainting_problem
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((1, 3, H, W), generator=g).to(DEV)
    if deblur:
        dg, y, init = deblurring_problem(x, seed_ip=0, l=2)
    else:
        dg, y, init, _, _ = inpainting_problem(x, seed_ip=0)
    return dg, init.repeat(B, 1, 1, 1).contiguous()


@pytest.mark.parametrize("alpha", [1.0, 0.6])
def test_relax_langevin_inpaint_equals_unfused(alpha):
    from psgla_for_posterior_sampling_amd import hip_ops as K
    dg, _ = problem(B=3)
    B, C, H, W = 3, 3, 32, 48
    g = torch.Generator(device=DEV).manual_seed(5)
    c1, c2, seed = 0.8 * (1 / 255.0) ** 2, 0.011, 7
    sched_a = K.Schedule((B, C, H, W), 12, 3, 2, DEV)
    sched_b = K.Schedule((B, C, H, W), 12, 3, 2, DEV)
    ma, qa = torch.zeros(B, C, H, W, device=DEV), torch.zeros(B, C, H, W, device=DEV)
    mb, qb = ma.clone(), qa.clone()
    for i in range(12):
        Y = torch.rand((B, C, H, W), generator=g, device=DEV)
        D = torch.rand((B, C, H, W), generator=g, device=DEV)
        Yn_a = torch.empty_like(Y)
        Xa = torch.empty_like(Y)
        K.relax_langevin_inpaint(Y, D, alpha, dg.y, dg.mask_u8, dg.sigma2, c1, c2, seed, 4, ma, qa, sched_a, i, Yn_a,
                                 X_out=Xa)
        Xb = K.relax_accumulate(Y, D, torch.empty_like(Y), alpha, mb, qb, sched_b, i)
        gr = K.inpaint_grad(Xb, dg.y, dg.mask_u8, dg.sigma2)
        Yn_b = K.langevin_update(Xb, gr, c1, c2, seed, 4, i + 1)
        torch.cuda.synchronize()
        assert torch.equal(Xa, Xb)
        assert torch.equal(Yn_a, Yn_b)
        assert torch.equal(ma, mb) and torch.equal(qa, qb)
    assert torch.equal(sched_a.samples, sched_b.samples)
    assert torch.equal(sched_a.blocks, sched_b.blocks) and torch.equal(sched_a.blocks2, sched_b.blocks2)


@pytest.mark.parametrize("deblur,alpha", [(False, 1.0), (False, 0.5), (True, 1.0)])
def test_denoiser_chains_graph_equals_step_loop(deblur, alpha):
    """Typed fidelity + torch DnCNN -> DenoiserChains (hipGraph replay) == the generic step-by-step loop."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    dg, init = problem(deblur=deblur)
    den = small_dncnn().to(DEV)
    s = 2 / 255.0
    kw = dict(sig_float=s, delta=6.1515e-5, n_iter=40, n_inter=4, n_inter_mmse=4, seed=3)
    a = RA.psgla(init, dg, den, torch.tensor(alpha), torch.tensor(5.0), graph_steps=8, **kw)
    b = RA.psgla(init, lambda x: dg(x), den, torch.tensor(alpha), torch.tensor(5.0), **kw)   # opaque closure
    for la, lb in zip(a, b):
        assert len(la) == len(lb) > 0
        for u, v in zip(la, lb):
            assert torch.equal(u, v)


def test_denoiser_chains_vs_oracle():
    """GPU DnCNN path vs the CPU oracle (reference loop restated) with the same weights."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    dg, init = problem(B=1)
    den = small_dncnn()
    s = 2 / 255.0
    kw = dict(sig_float=s, delta=6.1515e-5, n_iter=30, n_inter=5, n_inter_mmse=5, seed=11)
    out = RA.psgla(init, dg, den.to(DEV), torch.tensor(1.0), torch.tensor(5.0), graph_steps=6, **kw)
    mask4 = torch.ones(3)[None, :, None, None] * dg.mask_u8.cpu().long()[None, None]
    y = dg.y.cpu()
    sig2 = torch.tensor(dg.sigma2, dtype=torch.float32)
    ref = orc.psgla(init.cpu(), lambda x: -mask4 * (x - y) / sig2, den.cpu(), torch.tensor(1.0), torch.tensor(5.0),
                    **kw)
    M = np.stack([t.cpu().numpy() for t in out[1]]).mean(0)
    Mr = np.stack([t.numpy() for t in ref[1]]).mean(0)
    assert rel(M, Mr) < REL_TOL_MEAN


@pytest.mark.parametrize("H,W,deblur", [(32, 48, False), (37, 45, False), (36, 45, False), (32, 48, True)])
def test_ula_chains_graph_equals_step_loop(H, W, deblur):
    """pnpula with a DenoiserPrior (DRUNet/DnCNN prior of sampling_images.py:156-157): UlaChains
    (hipGraph replay, the prior's arithmetic + data term + update fused in one V-ULA pass,
    pnpula_prior_update) == the step-by-step loop with the prior as an opaque closure (DenoiserPrior's
    torch ops, the data-term kernel, pnpula_update), bit for bit: inpainting on 4-aligned and odd planes
    (36 x 45: H*W % 4 == 0 with W % 4 != 0, the row-quad noise of psgla noise v2),
    deblurring (the stencil's gd fed to the fused pass)."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.denoisers import DenoiserPrior
    dg, init = problem(H=H, W=W, deblur=deblur)
    den = small_dncnn(seed=2).to(DEV)
    s1 = 5 / 255.0
    prior = DenoiserPrior(den, s1, torch.tensor(1.0, device=DEV), torch.tensor(s1 ** 2, device=DEV))
    kw = dict(delta=torch.tensor(1e-6), lambd=torch.tensor(3.7e-6), n_iter=30, n_inter=3, n_inter_mmse=3, seed=9)
    a = RA.pnpula(init, dg, prior, graph_steps=6, **kw)
    b = RA.pnpula(init, lambda x: dg(x), lambda x: prior(x), **kw)
    for la, lb in zip(a, b):
        assert len(la) == len(lb) > 0
        for u, v in zip(la, lb):
            assert torch.equal(u, v)


def test_drunet_forward_on_gpu():
    from psgla_for_posterior_sampling_amd.denoisers import DRUNet
    torch.manual_seed(0)
    m = DRUNet(nc=(16, 32, 64, 128), nb=1).to(DEV)
    x = torch.rand(2, 3, 40, 56, device=DEV)
    with torch.no_grad():
        y = m(x, 5 / 255.0)
        yc = m.cpu()(x.cpu(), 5 / 255.0)
    assert y.shape == x.shape
    assert rel(y.cpu().numpy(), yc.numpy()) < 1e-4


def test_denoiser_chains_independent_of_batch_split():
    """Chains keyed by global id (chain0): a 4-chain run == two 2-chain runs (multi-GPU sharding)."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    dg, init = problem(B=4)
    g = torch.Generator(device=DEV).manual_seed(8)
    init = (init + 0.05 * torch.rand(init.shape, generator=g, device=DEV)).contiguous()
    den = small_dncnn(seed=4).to(DEV)
    kw = dict(sig_float=2 / 255.0, delta=6.1515e-5, n_iter=20, n_inter=5, n_inter_mmse=4, seed=3, graph_steps=4)
    full = RA.psgla(init, dg, den, torch.tensor(1.0), torch.tensor(5.0), **kw)
    lo = RA.psgla(init[:2].contiguous(), dg, den, torch.tensor(1.0), torch.tensor(5.0), chain0=0, **kw)
    hi = RA.psgla(init[2:].contiguous(), dg, den, torch.tensor(1.0), torch.tensor(5.0), chain0=2, **kw)
    for f, a, b in zip(full, lo, hi):
        for u, v, w in zip(f, a, b):
            assert torch.equal(u, torch.cat([v, w], 0))


@pytest.mark.parametrize("channels_last", [True, False])
@pytest.mark.parametrize("relu", [True, False])
def test_bias_act_bitwise_vs_torch(channels_last, relu):
    """hip_ops.bias_act_ (the DnCNN layer epilogue) == PyTorch's bias add (+ ReLU), bit for bit,
    NHWC and NCHW, including zeros, negative zeros and large values."""
    from psgla_for_posterior_sampling_amd import hip_ops as K
    g = torch.Generator(device=DEV).manual_seed(3)
    y = torch.randn((3, 64, 20, 28), generator=g, device=DEV) * 5
    y[0, :, 0, :4] = 0.0
    y[1, :, 1, :4] = -0.0
    b = torch.randn(64, generator=g, device=DEV)
    b[:8] = 0.0
    if channels_last:
        y = y.contiguous(memory_format=torch.channels_last)
    ref = y + b.view(1, -1, 1, 1)
    if relu:
        ref = torch.relu(ref)
    out = K.bias_act_(y.clone(memory_format=torch.preserve_format), b, relu=relu)
    assert torch.equal(out, ref)
    assert torch.equal(torch.signbit(out), torch.signbit(ref))


def test_dncnn_fused_epilogue_equals_torch_layers():
    """DnCNN forward with the HIP bias+ReLU epilogue vs the same module run layer by layer in
    PyTorch (conv with bias, then ReLU) on the GPU.  Not bitwise: MIOpen may pick another solver
    (another summation order) for a convolution without bias, so fp32 tolerance."""
    from psgla_for_posterior_sampling_amd.denoisers import DnCNN
    torch.manual_seed(1)
    m = DnCNN(depth=6, device=DEV)
    x = torch.rand(2, 3, 32, 40, device=DEV)
    with torch.no_grad():
        out = m(x)
        xc = x.contiguous(memory_format=torch.channels_last)
        h = m.nl_list[0](m.in_conv(xc))
        for i in range(m.depth - 2):
            h = m.nl_list[i + 1](m.conv_list[i](h))
        ref = (m.out_conv(h) + xc).contiguous()
    assert rel(out.cpu().numpy(), ref.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("alpha", [1.0, 0.6])
@pytest.mark.parametrize("H,W", [(37, 45), (36, 45)])
def test_relax_langevin_inpaint_odd_plane_equals_unfused(alpha, H, W):
    """W % 4 != 0 (set1c / CBSD68 are 481 x 321): the row-quad variant of the fused pass equals
    relax_accumulate + inpaint_grad + langevin_update bit for bit -- also where H*W % 4 == 0 but W % 4 != 0
    (36 x 45), which the vector pass's plane-linear quads must not take (psgla noise v2 quads follow the rows)."""
    from psgla_for_posterior_sampling_amd import hip_ops as K
    B, C = 2, 3
    dg, _ = problem(B=B, H=H, W=W)
    g = torch.Generator(device=DEV).manual_seed(6)
    c1, c2, seed = 0.8 * (1 / 255.0) ** 2, 0.011, 9
    sched_a = K.Schedule((B, C, H, W), 8, 3, 2, DEV)
    sched_b = K.Schedule((B, C, H, W), 8, 3, 2, DEV)
    ma, qa = torch.zeros(B, C, H, W, device=DEV), torch.zeros(B, C, H, W, device=DEV)
    mb, qb = ma.clone(), qa.clone()
    for i in range(8):
        Y = torch.rand((B, C, H, W), generator=g, device=DEV)
        D = torch.rand((B, C, H, W), generator=g, device=DEV)
        Yn_a, Xa = torch.empty_like(Y), torch.empty_like(Y)
        K.relax_langevin_inpaint(Y, D, alpha, dg.y, dg.mask_u8, dg.sigma2, c1, c2, seed, 2, ma, qa, sched_a, i, Yn_a,
                                 X_out=Xa)
        Xb = K.relax_accumulate(Y, D, torch.empty_like(Y), alpha, mb, qb, sched_b, i)
        Yn_b = K.langevin_update(Xb, K.inpaint_grad(Xb, dg.y, dg.mask_u8, dg.sigma2), c1, c2, seed, 2, i + 1)
        torch.cuda.synchronize()
        assert torch.equal(Xa, Xb) and torch.equal(Yn_a, Yn_b)
        assert torch.equal(ma, mb) and torch.equal(qa, qb)
    assert torch.equal(sched_a.samples, sched_b.samples) and torch.equal(sched_a.blocks, sched_b.blocks)


def test_denoiser_chains_odd_plane_graph_equals_step_loop():
    """Config 3 on a 481 x 321-like plane (here 37 x 45: H*W odd): DenoiserChains runs hipGraph-captured
    and equals the generic step-by-step loop bit for bit."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    dg, init = problem(B=2, H=37, W=45)
    den = small_dncnn().to(DEV)
    kw = dict(sig_float=2 / 255.0, delta=6.1515e-5, n_iter=30, n_inter=3, n_inter_mmse=4, seed=5)
    a = RA.psgla(init, dg, den, torch.tensor(1.0), torch.tensor(5.0), graph_steps=6, **kw)
    b = RA.psgla(init, lambda x: dg(x), den, torch.tensor(1.0), torch.tensor(5.0), **kw)
    for la, lb in zip(a, b):
        assert len(la) == len(lb) > 0
        for u, v in zip(la, lb):
            assert torch.equal(u, v)


def _check_snapshots(path, name, n_iter, lists, extra_keys, with_y, B):
    import os
    K_ = n_iter // 10
    files = sorted(os.listdir(path))
    xs = sorted(f for f in files if f.startswith("x_"))
    assert xs == sorted(f"x_{i}.png" for i in range(0, n_iter, K_))
    ys = sorted(f for f in files if f.startswith("y_"))
    assert ys == (sorted(f"y_{i}.png" for i in range(0, n_iter, K_)) if with_y else [])
    d = torch.load(os.path.join(path, name + "_sampling.pth"), weights_only=True)   # our own output file
    assert set(d) == {"Samples", "Mmse", "Mmse2", "n_iter"} | set(extra_keys)
    # the last snapshot was taken after step i_last: the lists as they stood then
    i_last = ((n_iter - 1) // K_) * K_
    for key, full in zip(("Samples", "Mmse", "Mmse2"), lists):
        assert 0 < len(d[key]) <= len(full)
        for u, v in zip(d[key], full):
            assert torch.equal(u, v)
    return i_last


@pytest.mark.parametrize("den_kind", ["tv", "dncnn", "ula"])
def test_save_images_online_keeps_the_fast_path(tmp_path, den_kind):
    """save_images_online (restoration_algorithms.py:246-253, :273-283; :124-127, :146-158) on the
    engines themselves: the returned lists equal the run without snapshots bit for bit, x_i / y_i PNGs
    exist for exactly i % (n_iter / 10) == 0, and the saved dict has the reference's keys with the lists
    as they stood at the last snapshot."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.denoisers import DenoiserPrior, TVDenoiser
    B, n = 3, 40
    dg, init = problem(B=B, H=24, W=40)
    path = str(tmp_path)
    if den_kind == "ula":
        den = small_dncnn().to(DEV)
        prior = DenoiserPrior(den, 5 / 255.0 / 255.0, torch.tensor(1.0, device=DEV),
                              torch.tensor((5 / 255.0 / 255.0) ** 2, device=DEV))
        kw = dict(n_iter=n, n_inter=3, n_inter_mmse=4, seed=4, graph_steps=4)
        delta = torch.tensor(1e-6, device=DEV)
        a = RA.pnpula(init, dg, prior, delta, torch.tensor(1e-5), **kw)
        b = RA.pnpula(init, dg, prior, delta, torch.tensor(1e-5), path=path, save_images_online=True, name="nm",
                      **kw)
        extra, with_y = ("c_min", "c_max", "lambda", "delta"), False
    else:
        if den_kind == "tv":
            s, lam, mk = 10 / 255.0, 10.0, (lambda: TVDenoiser(n_it_max=10, exact=True))
        else:
            s, lam, mk = 2 / 255.0, 5.0, (lambda: small_dncnn().to(DEV))
        kw = dict(sig_float=s, delta=s ** 2, n_iter=n, n_inter=3, n_inter_mmse=4, seed=4, graph_steps=4)
        a = RA.psgla(init, dg, mk(), torch.tensor(1.0), torch.tensor(lam), **kw)
        b = RA.psgla(init, dg, mk(), torch.tensor(1.0), torch.tensor(lam), path=path, save_images_online=True,
                     name="nm", **kw)
        assert torch.isfinite(torch.stack(a[1])).all()
        extra, with_y = ("lambda", "delta"), True
    for la, lb in zip(a, b):
        assert len(la) == len(lb) > 0
        for u, v in zip(la, lb):
            assert torch.equal(u, v)
    i_last = _check_snapshots(path, "nm", n, b, extra, with_y, B)
    d = torch.load(path + "/nm_sampling.pth", weights_only=True)
    assert len(d["Samples"]) == i_last // 3 + 1          # samples at i % n_inter == 0, i <= i_last
    assert len(d["Mmse"]) == (i_last + 1) // 5           # blocks of n_inter_mmse + 1 steps completed
    assert d["n_iter"] == n


@pytest.mark.parametrize("exact", [True, False])
def test_save_images_online_y_matches_oracle(tmp_path, exact):
    """The y_i.png image of the fused TV path (restoration_algorithms.py:246-253: Y of step i, the input of
    the prox) is rebuilt after the step from X_i by the standalone inpaint_grad + langevin_update kernels;
    it equals the oracle's Y at step i (the tensor its psgla hands to denoiser.forward) bit for bit when the
    kernels run in exact mode, within the 1e-5 relative north-star tolerance in fast mode (the rebuild reads the fast chain's X_i)."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.denoisers import TVDenoiser
    from psgla_for_posterior_sampling_amd.fidelity import InpaintingFidelity
    g = torch.Generator().manual_seed(2)
    x = torch.rand((1, 3, 24, 40), generator=g)
    dg_ref, y, init, mask2d = orc.inpainting_problem(x, seed_ip=0)
    dg = InpaintingFidelity(mask2d.to(DEV), y.to(DEV), torch.tensor((1 / 255.0) ** 2, dtype=torch.float32))
    s, lam, n = 10 / 255.0, 10.0, 30
    kw = dict(sig_float=s, delta=s ** 2, n_iter=n, n_inter=3, n_inter_mmse=4, seed=4)

    class RecordingTV(orc.TVDenoiser):
        def __init__(self):
            super().__init__(n_it_max=10)
            self.ys = []

        def forward(self, y_in, ths=None):
            self.ys.append(y_in.clone())
            return super().forward(y_in, ths)
    tv = RecordingTV()
    orc.psgla(init, dg_ref, tv, torch.tensor(1.0), torch.tensor(lam), chain=0, **kw)

    seen = {}
    orig = RA._Snapshots.save

    def save(self, i, X, Y, lists):
        seen[i] = Y.detach().cpu().clone()
        return orig(self, i, X, Y, lists)
    RA._Snapshots.save = save
    try:
        RA.psgla(init.to(DEV), dg, TVDenoiser(n_it_max=10, exact=exact), torch.tensor(1.0), torch.tensor(lam),
                 path=str(tmp_path), save_images_online=True, name="nm", graph_steps=4, **kw)
    finally:
        RA._Snapshots.save = orig
    assert sorted(seen) == list(range(0, n, n // 10))
    for i, Yi in seen.items():
        if exact:
            assert torch.equal(Yi, tv.ys[i]), i
        else:
            d = float(torch.linalg.vector_norm((Yi - tv.ys[i]).double()) / torch.linalg.vector_norm(tv.ys[i].double()))
            assert d < REL_TOL_MEAN, (i, d)
        assert os.path.exists(os.path.join(str(tmp_path), f"y_{i}.png"))


def test_tv_prox_long_n_it_chunked_vs_oracle():
    """n_it_max = 30 > PSGLA_TV_MAX_FUSED_IT: the prox runs as two chunks (24 + 6 inner iterations) and is
    bit-identical to deepinv's loop (oracle), cold and warm-started, with and without an early stop."""
    from psgla_for_posterior_sampling_amd.denoisers import TVDenoiser
    g = torch.Generator().manual_seed(3)
    y = torch.rand((1, 3, 20, 28), generator=g)
    for tol in (1e-5, 2e-3):                    # 2e-3: deepinv stops inside the first chunk or the second
        ref = orc.TVDenoiser(n_it_max=30, tol=tol)
        den = TVDenoiser(n_it_max=30, tol=tol, exact=True)
        for call in range(3):
            yy = y + 0.02 * call
            r = ref.forward(yy, 0.05)
            o = den.forward(yy.to(DEV), 0.05)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(o.cpu().numpy(), r.numpy(), err_msg=f"tol {tol} call {call}")
            np.testing.assert_array_equal(den.u2.cpu().numpy(), ref.u2.numpy())


def test_tv_prox_per_chain_early_stop_equals_single_chain_calls():
    """per_chain=True on a batch of chains == one call per chain (deepinv's whole-tensor norm per chain),
    including one chain that early-stops while the others do not."""
    from psgla_for_posterior_sampling_amd.denoisers import TVDenoiser
    g = torch.Generator().manual_seed(4)
    y = torch.rand((3, 3, 18, 26), generator=g)
    y[1] = 0.5 + 0.001 * y[1]                 # nearly flat: converges (stops) within a few iterations
    for n_it in (10, 30):
        den = TVDenoiser(n_it_max=n_it, tol=1e-3, exact=True)
        singles = [TVDenoiser(n_it_max=n_it, tol=1e-3, exact=True) for _ in range(3)]
        for call in range(2):
            yy = (y + 0.01 * call).to(DEV)
            o = den.forward(yy, 0.05, per_chain=True)
            for b in range(3):
                ob = singles[b].forward(yy[b:b + 1].contiguous(), 0.05)
                assert torch.equal(o[b:b + 1], ob), (n_it, call, b)
                assert torch.equal(den.u2[b:b + 1], singles[b].u2)


def test_generic_tv_path_batch_equals_fused():
    """A B > 1 TV run through the generic loop (opaque data_grad closure) equals the fused kernel's run:
    per-chain early stop on both paths (restoration_algorithms.py:238 called once per chain by the
    reference)."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.denoisers import TVDenoiser
    dg, init = problem(B=3, H=24, W=40)
    kw = dict(sig_float=10 / 255.0, delta=(10 / 255.0) ** 2, n_iter=20, n_inter=3, n_inter_mmse=4, seed=2)
    a = RA.psgla(init, dg, TVDenoiser(n_it_max=10, exact=True), torch.tensor(1.0), torch.tensor(10.0), **kw)
    b = RA.psgla(init, lambda x: dg(x), TVDenoiser(n_it_max=10, exact=True), torch.tensor(1.0), torch.tensor(10.0),
                 **kw)
    for la, lb in zip(a, b):
        for u, v in zip(la, lb):
            assert torch.equal(u, v)
