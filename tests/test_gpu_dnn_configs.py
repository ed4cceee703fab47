"""GPU tests of BASELINE configs 3-5 at their real operators: the composed engines (DenoiserChains,
UlaChains) with the full deepinv architectures (DnCNN depth 20 / nf 64, DRUNet nc 64-512 / nb 4; random
weights -- the reference's Pretrained_models/ is empty offline, so the denoiser arithmetic itself is parity
unpinned) against the CPU oracle running the SAME weights, and 64-chain 3 x 256 x 256 properties.

* config 4: PSGLA + DnCNN + 9 x 9 uniform circular deblurring (sampling_images.py:304-341, l = 4) at a CBSD68
  shape (2 chains of 321 x 481) vs oracle.psgla;
* config 3: PSGLA + DnCNN + inpainting at the castle orientation (481 x 321) vs oracle.psgla;
* config 5: PnP-ULA + DRUNet prior (sampling_images.py:147-168, restoration_algorithms.py:103-144) vs
  oracle.pnpula;
* each DNN config at 64 chains x 3 x 256 x 256: hipGraph replay == the generic step-by-step loop bit for bit,
  finite, and the block means consistent with the stored samples (restoration_algorithms.py:255-271).

The convolutions run in MIOpen on the GPU and in ATen on the CPU (other summation orders), so the oracle
comparisons use the north-star tolerance on the sample mean (REL_TOL_MEAN), not bit equality."""
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


def full_dncnn(seed=0):
    """deepinv DnCNN(depth=20, nf=64) with PyTorch's default (random) initialisation."""
    from psgla_for_posterior_sampling_amd.denoisers import DnCNN
    torch.manual_seed(seed)
    return DnCNN(depth=20, nf=64)


def full_drunet(seed=0):
    """deepinv DRUNet(nc=[64, 128, 256, 512], nb=4), random initialisation."""
    from psgla_for_posterior_sampling_amd.denoisers import DRUNet
    torch.manual_seed(seed)
    return DRUNet(nc=(64, 128, 256, 512), nb=4)


def images(B, H, W, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.rand((B, 3, H, W), generator=g)


def oracle_chains(run_one, B):
    """Run the oracle once per chain (each chain is one reference run, noise keyed by chain id) and stack."""
    outs = [run_one(b) for b in range(B)]
    return [[torch.cat([o[k][i][None] for o in outs], 0) for i in range(len(outs[0][k]))] for k in range(3)]


def mean_of_blocks(blocks):
    return np.stack([t.detach().cpu().numpy() for t in blocks]).mean(0)


def test_config4_dncnn_deblur_9x9_cbsd68_shape_vs_oracle():
    """Config 4: DenoiserChains + BlurFidelity (l = 4 uniform, 9 x 9 circular) + depth-20 DnCNN, 2 chains of
    321 x 481 (CBSD68's majority orientation), DnCNN constants (s = 2/255, lambda = 5, delta = s^2), vs
    oracle.psgla with the reference's conv2d-based A / A^T and the same weights."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.engine import DenoiserChains  # noqa: F401  (the path under test)
    from psgla_for_posterior_sampling_amd.fidelity import BlurFidelity, deblurring_problem
    B, H, W, n = 2, 321, 481, 10
    x = images(1, H, W)
    dg_ref, y_ref, init_ref = orc.deblurring_problem(x, seed_ip=0, l=4)
    dg, y, init = deblurring_problem(x.to(DEV), seed_ip=0, l=4)
    assert isinstance(dg, BlurFidelity)
    # the same observation on both sides (the device generator's noise differs from the CPU one)
    dg.y = y_ref.to(DEV)
    init = y_ref.to(DEV).repeat(B, 1, 1, 1).contiguous()
    den = full_dncnn(seed=3)
    s = 2 / 255.0
    kw = dict(sig_float=s, delta=s ** 2, n_iter=n, n_inter=2, n_inter_mmse=2, seed=7)
    out = RA.psgla(init, dg, den.to(DEV), torch.tensor(1.0), torch.tensor(5.0), graph_steps=4, **kw)
    den_cpu = full_dncnn(seed=3)
    ref = oracle_chains(lambda b: orc.psgla(y_ref.clone(), dg_ref, den_cpu, torch.tensor(1.0), torch.tensor(5.0),
                                            chain=b, **kw), B)
    assert len(out[1]) == len(ref[1]) == n // 3
    for b in range(B):
        M = mean_of_blocks([t[b] for t in out[1]])
        Mr = mean_of_blocks([t[b] for t in ref[1]])
        assert np.isfinite(M).all()
        assert rel(M, Mr) < REL_TOL_MEAN, (b, rel(M, Mr))
        S = np.stack([t[b].cpu().numpy() for t in out[0]])
        Sr = np.stack([t[b].numpy() for t in ref[0]])
        assert rel(S, Sr) < 1e-4


def test_config3_dncnn_inpaint_castle_shape_vs_oracle():
    """Config 3: DenoiserChains + InpaintingFidelity + depth-20 DnCNN on one 481 x 321 chain (castle's shape,
    the reference's batch-1 run) vs oracle.psgla with the same weights and mask."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.fidelity import InpaintingFidelity
    H, W, n = 481, 321, 10
    x = images(1, H, W, seed=2)
    dg_ref, y, init, mask2d = orc.inpainting_problem(x, seed_ip=0)
    dg = InpaintingFidelity(mask2d.to(DEV), y.to(DEV), torch.tensor((1 / 255.0) ** 2, dtype=torch.float32))
    den = full_dncnn(seed=5)
    s = 2 / 255.0
    kw = dict(sig_float=s, delta=s ** 2, n_iter=n, n_inter=2, n_inter_mmse=2, seed=11)
    out = RA.psgla(init.to(DEV), dg, den.to(DEV), torch.tensor(1.0), torch.tensor(5.0), graph_steps=4, **kw)
    ref = orc.psgla(init, dg_ref, full_dncnn(seed=5), torch.tensor(1.0), torch.tensor(5.0), **kw)
    M, Mr = mean_of_blocks(out[1]), mean_of_blocks(ref[1])
    assert np.isfinite(M).all()
    assert rel(M, Mr) < REL_TOL_MEAN, rel(M, Mr)


@pytest.mark.parametrize("deblur", [False, True])
def test_config5_drunet_pnpula_vs_oracle(deblur):
    """Config 5: pnpula with the DRUNet prior of sampling_images.py:156-157 (s = 5 -> s1 = 5/255,
    lambda = 0.5 / (2/sigma^2 + alpha/s1^2), delta = 1/3 / (1/sigma^2 + 1/lambda + alpha/s1^2), [-1, 2]
    projection) through UlaChains vs oracle.pnpula with the same DRUNet weights, 2 chains of 64 x 96 (the
    U-Net's direct branch) -- inpainting (the configuration) and deblurring."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.denoisers import DenoiserPrior
    from psgla_for_posterior_sampling_amd.fidelity import InpaintingFidelity, deblurring_problem
    B, H, W, n = 2, 64, 96, 12
    x = images(1, H, W, seed=4)
    sigma2 = torch.tensor((1 / 255.0) ** 2, dtype=torch.float32)
    if deblur:
        dg_ref, y, init1 = orc.deblurring_problem(x, seed_ip=0, l=4)
        dg, _, _ = deblurring_problem(x.to(DEV), seed_ip=0, l=4)
        dg.y = y.to(DEV)
    else:
        dg_ref, y, init1, mask2d = orc.inpainting_problem(x, seed_ip=0)
        dg = InpaintingFidelity(mask2d.to(DEV), y.to(DEV), sigma2)
    s1 = 5 / 255.0
    alpha = torch.tensor(1.0)
    s2 = torch.tensor(s1 ** 2)
    lam = 0.5 / (2 / sigma2 + alpha / s1 ** 2)
    delta = 1 / 3 / (1 / sigma2 + 1 / lam + alpha / s1 ** 2)
    kw = dict(n_iter=n, n_inter=3, n_inter_mmse=2, seed=13)
    prior = DenoiserPrior(full_drunet(seed=6).to(DEV), s1, alpha.to(DEV), s2.to(DEV))
    init = init1.to(DEV).repeat(B, 1, 1, 1).contiguous()
    out = RA.pnpula(init, dg, prior, delta, lam, graph_steps=4, **kw)
    prior_cpu = DenoiserPrior(full_drunet(seed=6), s1, alpha, s2)
    ref = oracle_chains(lambda b: orc.pnpula(init1.clone(), dg_ref, prior_cpu, delta, lam, chain=b, **kw), B)
    assert len(out[1]) == len(ref[1]) == n // 3
    for b in range(B):
        M = mean_of_blocks([t[b] for t in out[1]])
        Mr = mean_of_blocks([t[b] for t in ref[1]])
        assert np.isfinite(M).all()
        assert rel(M, Mr) < REL_TOL_MEAN, (b, rel(M, Mr))


def _check_blocks_follow_samples(samples, blocks, blocks2, nm):
    """n_inter = 1: block k is the reference's running mean (restoration_algorithms.py:255-271, fp32) of the
    samples k (nm + 1) .. k (nm + 1) + nm; blocks2 the same of X ** 2."""
    for k in range(len(blocks)):
        m = torch.zeros_like(samples[0])
        q = torch.zeros_like(samples[0])
        for i in range(nm + 1):
            X = samples[k * (nm + 1) + i]
            m = i / (i + 1) * m + 1 / (i + 1) * X
            q = i / (i + 1) * q + 1 / (i + 1) * X ** 2
        torch.testing.assert_close(blocks[k], m, rtol=1e-6, atol=1e-7)
        torch.testing.assert_close(blocks2[k], q, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("workload", ["dncnn-inpaint", "dncnn-deblur", "drunet-ula"])
def test_dnn_config_64_chains_full_size_properties(workload):
    """64 chains x 3 x 256 x 256 (the bench shape) per DNN config: the hipGraph-replayed engine equals the
    step-by-step generic loop (the data term as an opaque closure) bit for bit, every output is finite, and
    the block means / second moments follow from the stored samples."""
    from psgla_for_posterior_sampling_amd import restoration_algorithms as RA
    from psgla_for_posterior_sampling_amd.denoisers import DenoiserPrior
    from psgla_for_posterior_sampling_amd.fidelity import deblurring_problem, inpainting_problem
    B, H, W, n, nm = 64, 256, 256, 12, 2
    g = torch.Generator(device=DEV).manual_seed(21)
    x = torch.rand((1, 3, H, W), generator=g, device=DEV)
    if workload == "dncnn-deblur":
        dg, y, init1 = deblurring_problem(x, seed_ip=0, l=4)
    else:
        dg, y, init1, _, _ = inpainting_problem(x, seed_ip=0)
    init = (init1.repeat(B, 1, 1, 1) + 0.01 * torch.rand((B, 3, H, W), generator=g, device=DEV)).contiguous()
    if workload == "drunet-ula":
        s1 = 5 / 255.0
        sigma2 = (1 / 255.0) ** 2
        lam = 0.5 / (2 / sigma2 + 1 / s1 ** 2)
        delta = 1 / 3 / (1 / sigma2 + 1 / lam + 1 / s1 ** 2)
        prior = DenoiserPrior(full_drunet(seed=8).to(DEV), s1, torch.tensor(1.0, device=DEV),
                              torch.tensor(s1 ** 2, device=DEV))
        kw = dict(n_iter=n, n_inter=1, n_inter_mmse=nm, seed=17)
        a = RA.pnpula(init, dg, prior, torch.tensor(delta), torch.tensor(lam), graph_steps=3, **kw)
        b = RA.pnpula(init, lambda t: dg(t), lambda t: prior(t), torch.tensor(delta), torch.tensor(lam), **kw)
    else:
        den = full_dncnn(seed=9).to(DEV)
        s = 2 / 255.0
        kw = dict(sig_float=s, delta=s ** 2, n_iter=n, n_inter=1, n_inter_mmse=nm, seed=17)
        a = RA.psgla(init, dg, den, torch.tensor(1.0), torch.tensor(5.0), graph_steps=3, **kw)
        b = RA.psgla(init, lambda t: dg(t), den, torch.tensor(1.0), torch.tensor(5.0), **kw)
    assert len(a[0]) == n and len(a[1]) == n // (nm + 1)
    for la, lb in zip(a, b):
        assert len(la) == len(lb) > 0
        for u, v in zip(la, lb):
            assert torch.equal(u, v)
    assert all(torch.isfinite(t).all() for t in a[0] + a[1] + a[2])
    _check_blocks_follow_samples(a[0], a[1], a[2], nm)
