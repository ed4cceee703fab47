"""GPU tests of the DNN-denoiser paths (BASELINE configs 3-5): the fused epilogue/prologue pass
(psgla_relax_langevin_inpaint), the hipGraph-replayed engines DenoiserChains / UlaChains against
the step-by-step generic loop (same kernels, same denoiser: bit for bit), and against the CPU
oracle (restoration_algorithms.py restated) within the north-star tolerance -- the convolutions
run in MIOpen on the GPU and in ATen on the CPU, so the denoiser itself is not bit-identical."""
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


def test_ula_chains_graph_equals_step_loop():
    """pnpula with a DenoiserPrior (DRUNet/DnCNN prior of sampling_images.py:156-157): UlaChains
    (hipGraph replay) == the step-by-step loop with the same prior as an opaque closure."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.denoisers import DenoiserPrior
    dg, init = problem()
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
