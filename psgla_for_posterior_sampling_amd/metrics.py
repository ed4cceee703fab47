"""Host-side metrics and the per-image result record of sampling_images.py:371-470.

PSNR and SSIM restate scikit-image 0.24's ``peak_signal_noise_ratio`` and
``structural_similarity`` with the arguments the reference passes (data_range=1, default
7x7 uniform window, sample covariance, K1=0.01, K2=0.03, mean over channel_axis=2).
scikit-image is not installed in this image, so the restatement is *parity unpinned*: it is
checked against closed-form cases and a direct evaluation in tests/test_metrics_cli.py, not
against skimage outputs; everything around PSNR / SSIM in ``analyse_run`` is pinned to the reference
sampling_images.py:371-442 executed on fixture outputs (tests/golden/postproc_inpaint_tv.npz).
"""
from __future__ import annotations

import numpy as np
from scipy.ndimage import uniform_filter


def _float_type(*arrays):
    # skimage's _supported_float_type: float32 stays float32, everything else -> float64
    return np.float32 if all(a.dtype == np.float32 for a in arrays) else np.float64


def psnr(image_true: np.ndarray, image_test: np.ndarray, data_range: float = 1.0) -> float:
    """skimage.metrics.peak_signal_noise_ratio (sampling_images.py:378, :399, :419)."""
    ft = _float_type(image_true, image_test)
    a = image_true.astype(ft, copy=False)
    b = image_test.astype(ft, copy=False)
    err = np.mean((a - b) ** 2, dtype=np.float64)
    return float(10 * np.log10((data_range ** 2) / err))


def _ssim_2d(X: np.ndarray, Y: np.ndarray, data_range: float, win_size: int = 7, K1: float = 0.01,
             K2: float = 0.03) -> float:
    NP = win_size ** 2
    cov_norm = NP / (NP - 1)
    ux = uniform_filter(X, size=win_size)
    uy = uniform_filter(Y, size=win_size)
    uxx = uniform_filter(X * X, size=win_size)
    uyy = uniform_filter(Y * Y, size=win_size)
    uxy = uniform_filter(X * Y, size=win_size)
    vx = cov_norm * (uxx - ux * ux)
    vy = cov_norm * (uyy - uy * uy)
    vxy = cov_norm * (uxy - ux * uy)
    C1 = (K1 * data_range) ** 2
    C2 = (K2 * data_range) ** 2
    A1, A2, B1, B2 = (2 * ux * uy + C1, 2 * vxy + C2, ux ** 2 + uy ** 2 + C1, vx + vy + C2)
    S = (A1 * A2) / (B1 * B2)
    pad = (win_size - 1) // 2
    return float(S[pad:S.shape[0] - pad, pad:S.shape[1] - pad].mean(dtype=np.float64))


def ssim(im1: np.ndarray, im2: np.ndarray, data_range: float = 1.0, channel_axis: int | None = None) -> float:
    """skimage.metrics.structural_similarity with the reference's arguments
    (sampling_images.py:379-382, :398, :420-423)."""
    ft = _float_type(im1, im2)
    a = im1.astype(ft, copy=False)
    b = im2.astype(ft, copy=False)
    if channel_axis is None:
        return _ssim_2d(a, b, data_range)
    a = np.moveaxis(a, channel_axis, -1)
    b = np.moveaxis(b, channel_axis, -1)
    return float(np.mean([_ssim_2d(a[..., c], b[..., c], data_range) for c in range(a.shape[-1])]))


def _hwc(t, grayscale: bool) -> np.ndarray:
    x = t.detach().cpu().numpy() if hasattr(t, "detach") else np.asarray(t)
    if grayscale:
        return x[0, 0] if x.ndim == 4 else (x[0] if x.ndim == 3 else x)
    if x.ndim == 4:
        x = x[0]
    return np.transpose(x, (1, 2, 0))


def analyse_run(im: np.ndarray, samples_t, mmse_t, mmse2_t, y_t, init_t, grayscale: bool = False):
    """The reference's post-processing of one restored image (sampling_images.py:371-438):
    per-sample PSNR / SSIM / min / max, the running-MMSE PSNR / SSIM curve (cumulative mean of
    the block means), the MMSE, its PSNR / SSIM, and the pixel std from the second moments.
    Returns (record, extras) where record has the keys of the reference's result dict
    (minus the run parameters) and extras holds the sample / block arrays."""
    ch = None if grayscale else 2
    Samples, Psnr_sample, SIM_sample, Min_sample, Max_sample = [], [], [], [], []
    for sample in samples_t:
        samp = _hwc(sample, grayscale)
        Psnr_sample.append(psnr(im, samp, data_range=1))
        SIM_sample.append(ssim(im, samp, data_range=1, channel_axis=ch))
        Samples.append(samp)
        Min_sample.append(np.min(samp))
        Max_sample.append(np.max(samp))
    Mmse = np.array([_hwc(m, grayscale) for m in mmse_t])
    Mmse2 = [_hwc(m, grayscale) for m in mmse2_t]
    y = _hwc(y_t, grayscale)
    psb = psnr(im, y, data_range=1)
    ssb = ssim(im, y, data_range=1, channel_axis=ch)
    n = len(Mmse)
    shape = (n,) + (1,) * (Mmse.ndim - 1)
    mean_list = np.cumsum(Mmse, axis=0) / np.arange(1, n + 1).reshape(shape)
    PSNR_list, SIM_list = [], []
    for i in range(1, n):
        PSNR_list.append(psnr(im, mean_list[i], data_range=1))
        SIM_list.append(ssim(im, mean_list[i], data_range=1, channel_axis=ch))
    xmmse = np.mean(Mmse, axis=0)
    pmmse = psnr(im, xmmse, data_range=1)
    smmse = ssim(im, xmmse, data_range=1, channel_axis=ch)
    xmmse2 = np.mean(np.array(Mmse2), axis=0)
    var = xmmse2 - xmmse ** 2
    var = var * (var >= 0) + 0 * (var < 0)
    std = np.sqrt(var)
    diff = np.abs(im - xmmse)
    init = _hwc(init_t, grayscale)
    record = {
        "PSNR_sample": Psnr_sample, "SIM_sample": SIM_sample, "PSNR_mmse": PSNR_list, "SIM_list": SIM_list,
        "observation": y, "init": init, "PSNR_y": psb, "SIM_y": ssb, "ground_truth": im, "MMSE": xmmse,
        "PSNR_MMSE": pmmse, "SIM_MMSE": smmse, "std": std, "diff": diff,
    }
    extras = {"Samples": Samples, "Mmse": list(Mmse), "Mmse2": Mmse2, "Min_sample": Min_sample,
              "Max_sample": Max_sample}
    return record, extras
