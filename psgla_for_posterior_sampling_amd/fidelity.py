"""Data-fidelity terms of the two inverse problems (sampling_images.py:283-341).

The reference builds anonymous closures ``data_grad = lambda x: ...``.  Here they are typed
callables with the same call signature (``data_grad(x) -> tensor``), so that ``psgla`` can
recognise them and fuse the gradient into its HIP step kernel; called directly they run the
HIP gradient kernel.  The one-time problem set-up (mask / observation synthesis) issues the
same torch calls, in the same order, on the same generator as the reference, so the mask and
observation are bit-identical to what the reference builds on the same device.
"""
from __future__ import annotations

import numpy as np
import torch

from . import hip_ops as K


class InpaintingFidelity:
    """g(x) = -mask * (x - y) / sigma2   (sampling_images.py:295).

    mask_2d: (H, W) or (B, H, W) 0/1 tensor (1 = observed pixel), broadcast over channels;
    y: (1, C, H, W) shared or (B, C, H, W) per chain; sigma2: fp32 divisor (sigma2t)."""

    def __init__(self, mask_2d: torch.Tensor, y: torch.Tensor, sigma2):
        self.mask_u8 = mask_2d.to(torch.uint8).contiguous()
        self.y = y.contiguous().float()
        self.sigma2 = float(np.float32(float(sigma2)))

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return K.inpaint_grad(x.contiguous(), self.y, self.mask_u8, self.sigma2)


def inpainting_problem(im_t: torch.Tensor, seed_ip: int = 0, prop: float = 0.5, sigma: float = 1.0):
    """Random-pixel inpainting set-up of sampling_images.py:285-302 on im_t's device.

    Returns (data_grad, y_t, init, mask_2d, mask) with data_grad an InpaintingFidelity."""
    dev = im_t.device
    sigma1 = sigma / 255.0
    sigma2t = torch.tensor(sigma1 ** 2, dtype=torch.float32, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed_ip)
    m = torch.rand((im_t.shape[2], im_t.shape[3]), generator=gen, device=dev)
    mask_2d = 1 * (m > prop)
    C = im_t.shape[1]
    mask = torch.ones(C, device=dev)[None, :, None, None] * mask_2d[None, None, :, :]
    neg_mask = 1 - mask
    y_t = mask * im_t + torch.normal(torch.zeros(*im_t.size(), device=dev),
                                     std=sigma1 * torch.ones(*im_t.size(), device=dev), generator=gen)
    init = mask * y_t + neg_mask * 0.5 * torch.ones(y_t.shape, device=dev)
    return InpaintingFidelity(mask_2d, y_t, sigma2t), y_t, init, mask_2d, mask


def blur_kernel(l: int = 4, blur_type: str = "uniform", si: float = 1.0) -> np.ndarray:
    """(2l+1)^2 kernel h^T h of sampling_images.py:306-313 (float64, normalised)."""
    if blur_type == "uniform":
        h = np.ones((1, 2 * l + 1))
    elif blur_type == "gaussian":
        h = np.array([[np.exp(-i ** 2 / (2 * si ** 2)) for i in range(-l, l + 1)]])
    else:
        raise ValueError(f"unknown blur_type {blur_type!r}")
    h = h / np.sum(h)
    return np.dot(h.T, h)


class BlurFidelity:
    """g(x) = -A^T(A x - y) / sigma2 with A = circular (2l+1)^2 depthwise convolution
    (sampling_images.py:329-338).  Calling it runs the HIP stencil kernel (psgla_blur_grad);
    psgla() fuses it with the Langevin update.  A / AT (torch conv2d, as the reference) are kept
    for the one-time observation synthesis y = A(x) + noise."""

    def __init__(self, hconv: torch.Tensor, hcorr: torch.Tensor, l: int, y: torch.Tensor | None, sigma2,
                 exact: bool = False):
        self.hconv, self.hcorr, self.l = hconv, hcorr, int(l)
        self.y = y
        self.sigma2t = torch.as_tensor(sigma2, dtype=torch.float32, device=hconv.device)
        self.sigma2 = float(self.sigma2t.item())
        self.exact = exact
        # the HIP kernel takes one (2l+1, 2l+1) tap set shared by all channels
        hc = hconv.reshape(-1, hconv.shape[-2], hconv.shape[-1])
        hr = hcorr.reshape(-1, hcorr.shape[-2], hcorr.shape[-1])
        if not (torch.equal(hc, hc[:1].expand_as(hc)) and torch.equal(hr, hr[:1].expand_as(hr))):
            raise ValueError("BlurFidelity: per-channel blur kernels must be identical")
        self.taps_conv = hc[0].float().cpu().numpy()        # host copies: launch arguments
        self.taps_corr = hr[0].float().cpu().numpy()

    def A(self, x):
        l = self.l
        return torch.nn.functional.conv2d(torch.nn.functional.pad(x, [l, l, l, l], mode="circular"),
                                          self.hconv, groups=x.size(1), padding=0)

    def AT(self, x):
        l = self.l
        return torch.nn.functional.conv2d(torch.nn.functional.pad(x, [l, l, l, l], mode="circular"),
                                          self.hcorr, groups=x.size(1), padding=0)

    def __call__(self, x):
        return K.blur_grad(x.contiguous(), self.y.contiguous(), self.taps_conv, self.taps_corr, self.l, self.sigma2,
                           exact=self.exact)


def deblurring_problem(im_t: torch.Tensor, seed_ip: int = 0, l: int = 4, blur_type: str = "uniform",
                       si: float = 1.0, sigma: float = 1.0):
    """Deblurring set-up of sampling_images.py:306-341.  Returns (data_grad, y_t, init)."""
    dev = im_t.device
    C = im_t.shape[1]
    sigma1 = sigma / 255.0
    sigma2t = torch.tensor(sigma1 ** 2, dtype=torch.float32, device=dev)
    h_ = blur_kernel(l, blur_type, si)
    hconv = torch.from_numpy(np.copy(np.flip(h_))).type(torch.FloatTensor).to(dev)
    hcorr = torch.from_numpy(h_).type(torch.FloatTensor).to(dev)
    ones = torch.ones(C, hconv.shape[0], hconv.shape[1], device=dev)
    hconv = hconv.unsqueeze(0)[None, :, :, :] * ones[:, None, :, :]
    hcorr = hcorr.unsqueeze(0)[None, :, :, :] * ones[:, None, :, :]
    fid = BlurFidelity(hconv, hcorr, l, None, sigma2t)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed_ip)
    y_t = fid.A(im_t) + torch.normal(torch.zeros(*im_t.size(), device=dev),
                                     std=sigma1 * torch.ones(*im_t.size(), device=dev), generator=gen)
    fid.y = y_t
    return fid, y_t, y_t
