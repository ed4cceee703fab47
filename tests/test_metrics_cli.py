"""Host metrics (metrics.py, a restatement of skimage's PSNR / SSIM: parity unpinned -- skimage is
not installed) and the CLI's parameter / path semantics (sampling_images.py:52-198)."""
import os

import numpy as np
import pytest

from psgla_for_posterior_sampling_amd import metrics
from psgla_for_posterior_sampling_amd import sampling_images as SI


def test_psnr_closed_form():
    a = np.zeros((8, 8, 3), np.float32)
    b = np.full((8, 8, 3), 0.1, np.float32)
    assert abs(metrics.psnr(a, b) - 20.0) < 1e-5          # mse = 0.01 -> 20 dB


def _ssim_naive(X, Y, R=1.0, w=7):
    """Direct float64 evaluation of skimage's default SSIM (uniform 7x7 window, reflect padding,
    sample covariance), pixel by pixel."""
    X = X.astype(np.float64)
    Y = Y.astype(np.float64)
    p = w // 2
    Xp = np.pad(X, p, mode="symmetric")
    Yp = np.pad(Y, p, mode="symmetric")
    H, W = X.shape
    S = np.zeros((H, W))
    C1, C2 = (0.01 * R) ** 2, (0.03 * R) ** 2
    for i in range(H):
        for j in range(W):
            x = Xp[i:i + w, j:j + w].ravel()
            y = Yp[i:i + w, j:j + w].ravel()
            ux, uy = x.mean(), y.mean()
            n = w * w
            vx = ((x * x).mean() - ux * ux) * n / (n - 1)
            vy = ((y * y).mean() - uy * uy) * n / (n - 1)
            vxy = ((x * y).mean() - ux * uy) * n / (n - 1)
            S[i, j] = ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux ** 2 + uy ** 2 + C1) * (vx + vy + C2))
    return S[p:H - p, p:W - p].mean()


def test_ssim_matches_direct_evaluation():
    rng = np.random.default_rng(0)
    x = rng.random((20, 23))
    y = np.clip(x + 0.1 * rng.standard_normal(x.shape), 0, 1)
    assert abs(metrics.ssim(x, y) - _ssim_naive(x, y)) < 1e-10
    assert abs(metrics.ssim(x, x) - 1.0) < 1e-12
    xc = rng.random((16, 18, 3))
    yc = rng.random((16, 18, 3))
    ref = np.mean([_ssim_naive(xc[..., c], yc[..., c]) for c in range(3)])
    assert abs(metrics.ssim(xc, yc, channel_axis=2) - ref) < 1e-10


def test_analyse_run_record_keys_and_values():
    import torch
    rng = np.random.default_rng(1)
    im = rng.random((12, 14, 3)).astype(np.float32)
    chw = lambda a: torch.from_numpy(np.ascontiguousarray(np.transpose(a, (2, 0, 1))))  # noqa: E731
    samples = [chw(np.clip(im + 0.05 * rng.standard_normal(im.shape).astype(np.float32), 0, 1)) for _ in range(4)]
    blocks = [chw(im + 0.01 * k) for k in range(3)]
    blocks2 = [chw((im + 0.01 * k) ** 2 + 0.001) for k in range(3)]
    y = chw(im)[None]
    rec, ex = metrics.analyse_run(im, samples, blocks, blocks2, y, y)
    for k in ("PSNR_sample", "SIM_sample", "PSNR_mmse", "SIM_list", "observation", "init", "PSNR_y", "SIM_y",
              "ground_truth", "MMSE", "PSNR_MMSE", "SIM_MMSE", "std", "diff"):
        assert k in rec
    assert len(rec["PSNR_sample"]) == 4 and len(rec["PSNR_mmse"]) == 2
    np.testing.assert_allclose(rec["MMSE"], im + 0.01, rtol=0, atol=1e-6)
    assert abs(rec["PSNR_MMSE"] - metrics.psnr(im, rec["MMSE"])) < 1e-12
    assert np.all(rec["std"] >= 0)


def _postproc_inputs(golden_dir):
    import torch
    z = np.load(os.path.join(golden_dir, "psgla_inpaint_tv.npz"))
    im = np.float32(np.transpose(z["x"][0], (1, 2, 0)))
    return (im, [torch.from_numpy(s) for s in z["samples"]], [torch.from_numpy(s) for s in z["blocks"]],
            [torch.from_numpy(s) for s in z["blocks2"]], torch.from_numpy(z["y"]), torch.from_numpy(z["init"]))


def test_analyse_run_matches_reference_postprocessing(golden_dir):
    """metrics.analyse_run against sampling_images.py:371-442 executed on the psgla+TV fixture's chain
    outputs (tests/golden/make_golden.py make_postproc, PSNR / ssim bound to metrics.*): every
    result-dict value is identical -- the curve over range(1, n), MMSE, std, diff, min / max, and the
    float32 / float64 types the reference's numpy expressions produce.  SSIM's own arithmetic stays
    parity unpinned (skimage absent)."""
    ref = np.load(os.path.join(golden_dir, "postproc_inpaint_tv.npz"))
    im, samples, blocks, blocks2, y, init = _postproc_inputs(golden_dir)
    rec, ex = metrics.analyse_run(im, samples, blocks, blocks2, y, init)
    for k in ("PSNR_sample", "SIM_sample", "PSNR_mmse", "SIM_list"):
        np.testing.assert_array_equal(np.array(rec[k], np.float64), ref[k], err_msg=k)
    for k in ("PSNR_y", "SIM_y", "PSNR_MMSE", "SIM_MMSE"):
        assert rec[k] == float(ref[k]), k
    for k in ("observation", "init", "MMSE", "std", "diff"):
        assert rec[k].dtype == ref[k].dtype, k
        np.testing.assert_array_equal(rec[k], ref[k], err_msg=k)
    np.testing.assert_array_equal(np.array(ex["Min_sample"]), ref["Min_sample"])
    np.testing.assert_array_equal(np.array(ex["Max_sample"]), ref["Max_sample"])


def test_parameters_follow_flag_presence():
    p = SI.build_parser()
    argv = ["--alg", "psgla", "--den", "TV"]
    N, s, lambd, delta, n_inter, _ = SI.algorithm_parameters(p.parse_args(argv), argv)
    assert (N, lambd, n_inter) == (1000, 10.0, 10) and abs(s - 10 / 255.) < 1e-15 and delta == s ** 2
    argv = ["--alg", "psgla", "--den", "TV", "--N", "10000", "--s", "10"]
    N, s, lambd, delta, n_inter, _ = SI.algorithm_parameters(p.parse_args(argv), argv)
    assert (N, n_inter) == (10000, 10)
    argv = ["--alg", "psgla", "--den", "DnCNN"]
    N, s, lambd, delta, n_inter, _ = SI.algorithm_parameters(p.parse_args(argv), argv)
    assert (N, lambd) == (10000, 5.0) and abs(s - 2 / 255.) < 1e-15
    argv = ["--alg", "pnp_ula", "--den", "DnCNN"]
    N, s, lambd, delta, n_inter, ex = SI.algorithm_parameters(p.parse_args(argv), argv)
    assert N == 100000 and abs(ex["s1"] - (2 / 255.) / 255.) < 1e-18     # the reference's s/255 quirk
    sigma2 = (1 / 255.) ** 2
    assert abs(lambd - 0.5 / (2 / sigma2 + 1 / ex["s2"])) < 1e-20
    with pytest.raises(NotImplementedError):
        argv = ["--alg", "red"]
        SI.algorithm_parameters(p.parse_args(argv), argv)


def test_result_path_scheme(tmp_path):
    p = SI.build_parser()
    argv = ["--alg", "psgla", "--den", "TV", "--prop", "0.5", "--N", "1000", "--results_root", str(tmp_path)]
    path = SI.result_path(p.parse_args(argv), argv)
    assert path == os.path.join(str(tmp_path), "images", "inpainting", "prop_0.5", "set1c", "psgla", "TV", "N_1000")
    assert os.path.isdir(path)


def test_cli_chain_ids_and_shape_batches(tmp_path):
    """Batched CLI bookkeeping (CPU): chain id = rank in the listing stably sorted by shape; batches hold
    images of one shape with consecutive chain ids, at most batch_size of them."""
    from PIL import Image
    d = tmp_path / "ds"
    d.mkdir()
    shapes = [(24, 32), (24, 32), (32, 24), (24, 32), (32, 24), (24, 32)]
    for i, (h, w) in enumerate(shapes):
        Image.fromarray(np.zeros((h, w, 3), np.uint8)).save(str(d / f"{i:03d}.png"))
    files = [str(d / f) for f in sorted(os.listdir(str(d)))]
    ids = SI.chain_ids(files)
    assert ids == [0, 1, 4, 2, 5, 3]
    assert SI.shape_batches(list(range(6)), files, ids, 2) == [[0, 1], [2, 4], [3, 5]]
    assert SI.shape_batches(list(range(6)), files, ids, 8) == [[0, 1, 3, 5], [2, 4]]
    assert SI.shape_batches([1, 2, 3], files, ids, 8) == [[1, 3], [2]]
