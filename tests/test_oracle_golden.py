"""Pin the CPU oracle (oracle/psgla_oracle.py, oracle/noise.c) against
(a) the published Philox4x32-10 known-answer vectors (Random123 kat_vectors) and
(b) the golden fixtures produced by the reference's own psgla/pnpula
    (tests/golden/make_golden.py).  Every comparison here is bit-exact."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import psgla_oracle as orc

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return dict(np.load(os.path.join(G, name + ".npz"), allow_pickle=False))


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    assert orc.philox4x32_10([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert orc.philox4x32_10([0xffffffff] * 4, [0xffffffff] * 2) == \
        [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert orc.philox4x32_10([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
                             [0xa4093822, 0x299f31d0]) == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_noise_is_standard_normal():
    z = orc.normal((1, 3, 256, 256), seed=0, chain=0, step=0).numpy().astype(np.float64).ravel()
    z = np.concatenate([z, orc.normal((1, 3, 256, 256), 0, 1, 0).numpy().ravel()])
    assert abs(z.mean()) < 4e-3
    assert abs(z.std() - 1) < 3e-3
    assert abs((z ** 4).mean() - 3) < 8e-2   # 5 sigma at n=393216
    from scipy import stats
    assert stats.kstest(z[:100000], "norm").pvalue > 1e-3


def test_noise_stream_independence():
    a = orc.normal((1, 3, 8, 8), 0, 0, 0)
    assert not torch.equal(a, orc.normal((1, 3, 8, 8), 0, 1, 0))   # chain
    assert not torch.equal(a, orc.normal((1, 3, 8, 8), 0, 0, 1))   # step
    assert not torch.equal(a, orc.normal((1, 3, 8, 8), 1, 0, 0))   # seed
    assert torch.equal(a, orc.normal((1, 3, 8, 8), 0, 0, 0))       # deterministic
    # element e of a larger image equals element e of a prefix (quad numbering)
    big = orc.normal((1, 3, 16, 16), 0, 0, 0).flatten()
    assert torch.equal(big[:192], orc.normal((1, 3, 8, 8), 0, 0, 0).flatten())


def test_radius_and_angle_tables_are_sane():
    r = orc.radius_table(0, 1 << 16)
    k = np.arange(1 << 16, dtype=np.float64)
    ref = np.sqrt(-2 * np.log((k + 1) * 2.0 ** -24))
    assert np.max(np.abs(r - ref) / ref) < 2e-6
    c, s = orc.angle_table(0, 1 << 20)
    th = 2 * np.pi * np.arange(1 << 20) * 2.0 ** -24
    assert np.max(np.abs(c - np.cos(th))) < 2e-7 and np.max(np.abs(s - np.sin(th))) < 2e-7


def _chk(out, fx, rtol=None):
    Xl, Ml, M2l = out
    for got, key in ((Xl, "samples"), (Ml, "blocks"), (M2l, "blocks2")):
        a = np.stack([t.numpy() for t in got])
        if rtol is None:
            np.testing.assert_array_equal(a, fx[key])
        else:
            np.testing.assert_allclose(a, fx[key], rtol=rtol, atol=rtol)


def test_inpainting_setup_matches_reference():
    fx = load("psgla_inpaint_clamp")
    dg, y, init, mask2d = orc.inpainting_problem(torch.from_numpy(fx["x"]), seed_ip=0)
    np.testing.assert_array_equal(y.numpy(), fx["y"])
    np.testing.assert_array_equal(init.numpy(), fx["init"])
    np.testing.assert_array_equal(mask2d.numpy().astype(np.uint8), fx["mask2d"])


def test_mask_256_bits():
    fx = load("mask_256_seed0")
    g = torch.Generator().manual_seed(0)
    m = (torch.rand((256, 256), generator=g) > 0.5).numpy().astype(np.uint8)
    np.testing.assert_array_equal(np.packbits(m), fx["mask_bits"])


def test_psgla_inpaint_clamp():
    fx = load("psgla_inpaint_clamp")
    seed, n, ni, nm, alpha, lam, s, delta = fx["meta"]
    dg, y, init, _ = orc.inpainting_problem(torch.from_numpy(fx["x"]), seed_ip=0)
    out = orc.psgla(init, dg, orc.ClampDenoiser(), torch.tensor(alpha, dtype=torch.float32),
                    torch.tensor(lam, dtype=torch.float32), sig_float=s, delta=delta, n_iter=int(n),
                    n_inter=int(ni), n_inter_mmse=int(nm), seed=int(seed))
    _chk(out, fx)


def test_psgla_inpaint_tv():
    fx = load("psgla_inpaint_tv")
    seed, n, ni, nm, alpha, lam, s, delta, ntv = fx["meta"]
    dg, y, init, _ = orc.inpainting_problem(torch.from_numpy(fx["x"]), seed_ip=3)
    np.testing.assert_array_equal(init.numpy(), fx["init"])
    tv = orc.TVDenoiser(n_it_max=int(ntv))
    out = orc.psgla(init, dg, tv, torch.tensor(alpha, dtype=torch.float32),
                    torch.tensor(lam, dtype=torch.float32), sig_float=s, delta=delta, n_iter=int(n),
                    n_inter=int(ni), n_inter_mmse=int(nm), seed=int(seed))
    _chk(out, fx)
    np.testing.assert_array_equal(tv.x2.numpy(), fx["tv_x2"])
    np.testing.assert_array_equal(tv.u2.numpy(), fx["tv_u2"])


@pytest.mark.parametrize("bt", ["uniform", "gaussian"])
def test_psgla_deblur(bt):
    fx = load(f"psgla_deblur_{bt}")
    seed, n, ni, nm, alpha, lam, s, delta, l = fx["meta"]
    dg, y, init = orc.deblurring_problem(torch.from_numpy(fx["x"]), seed_ip=0, l=int(l), blur_type=bt)
    np.testing.assert_array_equal(y.numpy(), fx["y"])
    np.testing.assert_array_equal(orc.blur_kernel(int(l), bt).astype(np.float32), fx["hcorr"])
    out = orc.psgla(init, dg, orc.ClampDenoiser(), torch.tensor(alpha, dtype=torch.float32),
                    torch.tensor(lam, dtype=torch.float32), sig_float=s, delta=delta, n_iter=int(n),
                    n_inter=int(ni), n_inter_mmse=int(nm), seed=int(seed))
    _chk(out, fx)


@pytest.mark.parametrize("bt,l", [("uniform", 4), ("gaussian", 2), ("uniform", 0)])
def test_blur_tap_order_restatement_matches_reference_closure(bt, l):
    """oracle.blur_grad_tap_order (the stencil's summation order, which pins the HIP kernel bit for
    bit) computes the reference closure -AT(A x - y) / sigma2 (sampling_images.py:329-338, here
    through the fixture's observation y) to fp32 rounding: |d| <= 2e-5 max|g|."""
    fx = load(f"psgla_deblur_{bt}")
    x = torch.from_numpy(fx["x"])
    dg, y, _ = orc.deblurring_problem(x, seed_ip=0, l=l, blur_type=bt)
    xs = (x + 0.05 * torch.randn(x.shape, generator=torch.Generator().manual_seed(1))).float()
    ref = dg(xs).numpy()
    h_ = orc.blur_kernel(l, bt)
    got = orc.blur_grad_tap_order(xs.numpy(), y.numpy(), np.flip(h_).astype(np.float32),
                                  h_.astype(np.float32), l, float(np.float32((1 / 255.0) ** 2)))
    assert got.dtype == np.float32
    assert np.abs(got - ref).max() <= 2e-5 * np.abs(ref).max()


def test_pnpula_inpaint_clamp():
    fx = load("pnpula_inpaint_clamp")
    seed, n, ni, nm, alpha, lam, s1, delta = fx["meta"]
    dg, y, init, _ = orc.inpainting_problem(torch.from_numpy(fx["x"]), seed_ip=0)
    s2t = torch.tensor(s1 ** 2, dtype=torch.float32)
    alphat = torch.tensor(alpha, dtype=torch.float32)
    den = orc.ClampDenoiser()
    out = orc.pnpula(init, dg, lambda x: alphat * (den.forward(x, s1) - x) / s2t,
                     torch.tensor(delta, dtype=torch.float32), torch.tensor(lam, dtype=torch.float32),
                     n_iter=int(n), n_inter=int(ni), n_inter_mmse=int(nm), seed=int(seed))
    _chk(out, fx)


def test_psgla_relaxation_alpha03():
    fx = load("psgla_inpaint_conv_alpha03")
    seed, n, ni, nm, alpha, lam, s, delta = fx["meta"]
    dg, y, init, _ = orc.inpainting_problem(torch.from_numpy(fx["x"]), seed_ip=4)
    den = orc.TinyConvDenoiser(torch.from_numpy(fx["weight"]), torch.from_numpy(fx["bias"]))
    out = orc.psgla(init, dg, den, torch.tensor(alpha, dtype=torch.float32),
                    torch.tensor(lam, dtype=torch.float32), sig_float=s, delta=delta, n_iter=int(n),
                    n_inter=int(ni), n_inter_mmse=int(nm), seed=int(seed))
    # torch's CPU conv2d (oneDNN) picks its accumulation order by host ISA, so the conv prior is
    # only reproducible to fp32 rounding across machines: north_star tolerance (1e-5 relative).
    _chk(out, fx, rtol=1e-5)


def test_reference_error_behaviour():
    x = torch.rand((1, 3, 8, 8))
    dg, y, init, _ = orc.inpainting_problem(x)
    with pytest.raises(ZeroDivisionError):   # K = int(n_iter/10) = 0
        orc.psgla(init, dg, orc.ClampDenoiser(), torch.tensor(1.0), torch.tensor(5.0), n_iter=5,
                  n_inter=1, n_inter_mmse=1, seed=0)
    with pytest.raises(UnboundLocalError):   # gen only exists when seed is given
        orc.psgla(init, dg, orc.ClampDenoiser(), torch.tensor(1.0), torch.tensor(5.0), n_iter=20,
                  n_inter=1, n_inter_mmse=1, seed=None)


def test_params_fixture_matches_survey_table():
    p = json.load(open(os.path.join(G, "params.json")))
    tv = p["psgla_TV_defaults"]
    assert tv["N"] == 1000 and tv["n_inter"] == 10 and tv["lambd"] == 10.0
    assert abs(tv["delta_float"] / tv["lambd"] / tv["sigma2t"] - 10.0) < 1e-4
    assert p["pnp_ula_DRUNet_N1e6"]["n_inter"] == 1000


def test_noise_v2_row_aligned_quads():
    """psgla noise v2 (oracle/noise.c): a chain's image is rows of W; element (row, col) takes output col & 3 of
    quad row * ceil(W/4) + col // 4, so a row's noise does not depend on W beyond its quad count -- an odd-width
    image equals the first W columns of the image padded to a multiple of 4 -- and W % 4 == 0 is the flat
    numbering (quad e // 4, output e % 4) of rounds 1-3 that the golden fixtures were made with."""
    for (c, h, w) in ((3, 5, 7), (1, 4, 5), (2, 3, 321), (1, 2, 1)):
        wq = (w + 3) // 4 * 4
        a = orc.normal((1, c, h, w), 11, 3, 17)
        b = orc.normal((1, c, h, wq), 11, 3, 17)
        assert torch.equal(a, b[..., :w])
    # row 1 of a 5-wide image starts a new quad (quad 2), unlike the flat numbering (element 5 = quad 1, output 1)
    z = orc.normal((1, 1, 2, 5), 0, 0, 0).flatten()
    q = orc.normal((1, 1, 1, 12), 0, 0, 0).flatten()       # quads 0, 1, 2 of the same stream
    assert torch.equal(z[5:9], q[8:12])
    assert torch.equal(z[:4], q[:4]) and z[4] == q[4]
