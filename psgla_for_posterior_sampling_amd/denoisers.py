"""Denoisers with deepinv 0.2.1's call protocol ``denoiser.forward(x, sigma)``.

* :class:`TVDenoiser` -- deepinv.models.TVDenoiser (constructed at sampling_images.py:138,
  called at restoration_algorithms.py:238) on the HIP TV-prox kernel: same constructor
  arguments, same warm-start state (``x2``, ``u2``, ``restart``), same early stop.
* :class:`DnCNN` -- deepinv.models.DnCNN architecture (sampling_images.py:130): 20 conv3x3
  layers, 64 features, ReLU, residual output; parameter names ``in_conv`` / ``conv_list.i`` /
  ``out_conv`` so a deepinv ``state_dict`` loads unchanged.  Runs on PyTorch-ROCm (MIOpen),
  as the north star prescribes for the DNN forward.
* :class:`DRUNet` -- deepinv.models.DRUNet architecture (sampling_images.py:136; KAIR's UNetRes):
  noise-level map as a 4th input channel, 4 scales (64/128/256/512 features), 4 residual blocks
  per scale, 2x2 strided-conv down / transposed-conv up, no biases.  Restated from the published
  deepinv 0.2.1 / KAIR layout (deepinv is not vendored in the reference and not installable
  here): module names follow that layout so a ``drunet_color.pth`` state_dict would load, but
  with neither the package nor the weights available its arithmetic is *parity unpinned*.
* :class:`DenoiserPrior` -- the PnP-ULA prior gradient of sampling_images.py:156-157,
  ``alpha * (D(x, s1) - x) / s2``, as a typed (capturable) callable.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import hip_ops as K


class TVDenoiser(torch.nn.Module):
    def __init__(self, verbose: bool = False, tau: float = 0.01, rho: float = 1.99, tol: float = 1e-5,
                 n_it_max: int = 1000, x2=None, u2=None, exact: bool = False):
        super().__init__()
        self.verbose = verbose
        self.n_it_max = n_it_max
        self.crit = tol
        self.restart = True
        self.tau = tau
        self.rho = rho
        self.sigma = 1 / self.tau / 8
        self.x2 = x2
        self.u2 = u2
        self.exact = exact           # True: bit-exact (reference op order, IEEE div/sqrt) kernels
        self._work = None

    def constants(self) -> K.TvConstants:
        return K.TvConstants(self.tau, self.rho, self.crit, self.n_it_max)

    def needs_restart(self, shape) -> bool:
        return self.restart or self.x2 is None or tuple(self.x2.shape) != tuple(shape)

    def forward(self, y, ths=None, per_chain: bool = False):
        """deepinv's forward.  per_chain=True (this build's extension, used by psgla over a batch of
        chains): the early stop is decided per chain -- each batch entry behaves as its own call --
        instead of on the whole tensor as deepinv does.  Any n_it_max: above
        PSGLA_TV_MAX_FUSED_IT the prox runs in chunks (hip_ops.tv_prox)."""
        if ths is None:
            raise TypeError("TVDenoiser.forward needs the threshold `ths` (the reference passes sigma)")
        y = y.contiguous()
        fresh = self.needs_restart(y.shape)
        k = self.constants()
        G = y.shape[0] if per_chain else 1
        it = min(max(k.n_it, 1), K.N.TV_MAX_FUSED_IT)
        if (self._work is None or self._work.norms.shape[0] < G or self._work.norms.shape[1] != it
                or self._work.norms.device != y.device):
            self._work = K.TvWorkspace(G, it, y.device)
        x2, u2 = K.tv_prox(y, float(ths), k, None if fresh else self.x2, None if fresh else self.u2,
                           fresh=fresh, exact=self.exact, work=self._work, per_chain=per_chain)
        self.x2, self.u2 = x2, u2
        self.restart = False
        return x2


class DnCNN(torch.nn.Module):
    """deepinv DnCNN(in_channels=3, out_channels=3, depth=20, nf=64, bias=True), residual."""

    def __init__(self, in_channels: int = 3, out_channels: int = 3, depth: int = 20, bias: bool = True,
                 nf: int = 64, pretrained: str | None = None, device="cpu", channels_last: bool = True):
        super().__init__()
        self.depth = depth
        # NHWC activations on the GPU: MIOpen's NHWC fp32 convolutions measured 7 % faster on the
        # 64 x 3 x 256 x 256 DnCNN forward (tools/bench_dnn.py); same fp32 arithmetic, other order
        self.channels_last = channels_last
        self.in_conv = torch.nn.Conv2d(in_channels, nf, kernel_size=3, stride=1, padding=1, bias=bias)
        self.conv_list = torch.nn.ModuleList(
            [torch.nn.Conv2d(nf, nf, kernel_size=3, stride=1, padding=1, bias=bias) for _ in range(depth - 2)])
        self.out_conv = torch.nn.Conv2d(nf, out_channels, kernel_size=3, stride=1, padding=1, bias=bias)
        self.nl_list = torch.nn.ModuleList([torch.nn.ReLU() for _ in range(depth - 1)])
        if pretrained is not None and os.path.exists(pretrained):
            sd = torch.load(pretrained, map_location="cpu", weights_only=True)
            self.load_state_dict(sd, strict=True)
        self.eval()
        self.to(device)

    def _conv_relu(self, conv, h, i):
        """relu(conv(h)).  On the GPU the bias add and the ReLU are one in-place HIP pass over the
        conv output (hip_ops.bias_act_: the same fp32 operations as PyTorch's bias add + ReLU, so the
        result is bit-identical) instead of two passes over a 64 x 64 x 256 x 256 activation."""
        # the HIP pass is invisible to autograd: used only when no gradient can flow through it
        no_grad = not torch.is_grad_enabled() or not (h.requires_grad or conv.weight.requires_grad
                                                      or conv.bias is None or conv.bias.requires_grad)
        if h.is_cuda and conv.bias is not None and isinstance(self.nl_list[i], torch.nn.ReLU) and no_grad:
            from . import hip_ops as K
            y = torch.nn.functional.conv2d(h, conv.weight, None, conv.stride, conv.padding)
            return K.bias_act_(y, conv.bias, relu=True)
        return self.nl_list[i](conv(h))

    def forward(self, x, sigma=None):
        nhwc = self.channels_last and x.is_cuda
        if nhwc:
            self.to(memory_format=torch.channels_last)
            x = x.contiguous(memory_format=torch.channels_last)
        x1 = self._conv_relu(self.in_conv, x, 0)
        for i in range(self.depth - 2):
            x1 = self._conv_relu(self.conv_list[i], x1, i + 1)
        out = self.out_conv(x1) + x
        return out.contiguous() if nhwc else out


class _ResBlock(torch.nn.Module):
    """x + conv3x3(relu(conv3x3(x))), no bias (KAIR ResBlock, mode 'CRC')."""

    def __init__(self, nc: int):
        super().__init__()
        self.res = torch.nn.Sequential(torch.nn.Conv2d(nc, nc, 3, 1, 1, bias=False), torch.nn.ReLU(inplace=True),
                                       torch.nn.Conv2d(nc, nc, 3, 1, 1, bias=False))

    def forward(self, x):
        return x + self.res(x)


class DRUNet(torch.nn.Module):
    """deepinv DRUNet(in_channels=3, out_channels=3, nc=[64, 128, 256, 512], nb=4, act_mode='R',
    downsample_mode='strideconv', upsample_mode='convtranspose')."""

    def __init__(self, in_channels: int = 3, out_channels: int = 3, nc=(64, 128, 256, 512), nb: int = 4,
                 pretrained: str | None = None, device="cpu", channels_last: bool = True):
        super().__init__()
        self.channels_last = channels_last      # NHWC activations on the GPU (see DnCNN)
        nn = torch.nn
        self.m_head = nn.Conv2d(in_channels + 1, nc[0], 3, 1, 1, bias=False)
        self.m_down1 = nn.Sequential(*[_ResBlock(nc[0]) for _ in range(nb)], nn.Conv2d(nc[0], nc[1], 2, 2, 0, bias=False))
        self.m_down2 = nn.Sequential(*[_ResBlock(nc[1]) for _ in range(nb)], nn.Conv2d(nc[1], nc[2], 2, 2, 0, bias=False))
        self.m_down3 = nn.Sequential(*[_ResBlock(nc[2]) for _ in range(nb)], nn.Conv2d(nc[2], nc[3], 2, 2, 0, bias=False))
        self.m_body = nn.Sequential(*[_ResBlock(nc[3]) for _ in range(nb)])
        self.m_up3 = nn.Sequential(nn.ConvTranspose2d(nc[3], nc[2], 2, 2, 0, bias=False), *[_ResBlock(nc[2]) for _ in range(nb)])
        self.m_up2 = nn.Sequential(nn.ConvTranspose2d(nc[2], nc[1], 2, 2, 0, bias=False), *[_ResBlock(nc[1]) for _ in range(nb)])
        self.m_up1 = nn.Sequential(nn.ConvTranspose2d(nc[1], nc[0], 2, 2, 0, bias=False), *[_ResBlock(nc[0]) for _ in range(nb)])
        self.m_tail = nn.Conv2d(nc[0], out_channels, 3, 1, 1, bias=False)
        if pretrained is not None and os.path.exists(pretrained):
            sd = torch.load(pretrained, map_location="cpu", weights_only=True)
            self.load_state_dict(sd, strict=True)
        self.eval()
        self.to(device)

    def forward_unet(self, x0):
        x1 = self.m_head(x0)
        x2 = self.m_down1(x1)
        x3 = self.m_down2(x2)
        x4 = self.m_down3(x3)
        x = self.m_body(x4)
        x = self.m_up3(x + x4)
        x = self.m_up2(x + x3)
        x = self.m_up1(x + x2)
        return self.m_tail(x + x1)

    def forward(self, x, sigma):
        if isinstance(sigma, torch.Tensor) and sigma.dim() > 0:
            nmap = sigma.view(-1, 1, 1, 1).to(x.dtype) * torch.ones((x.size(0), 1, x.size(2), x.size(3)),
                                                                      dtype=x.dtype, device=x.device)
        else:
            nmap = torch.full((x.size(0), 1, x.size(2), x.size(3)), float(sigma), dtype=x.dtype, device=x.device)
        x = torch.cat((x, nmap), 1)
        if self.channels_last and x.is_cuda:
            self.to(memory_format=torch.channels_last)
            x = x.contiguous(memory_format=torch.channels_last)
        return self._forward_dispatch(x).contiguous()

    def _forward_dispatch(self, x):
        """deepinv 0.2.1 DRUNet.forward's size dispatch (KAIR utils_model): the U-Net itself in eval mode
        when both sides are multiples of 8 and > 31; replicate padding to multiples of 16 (test_pad) in
        training mode or when a side is < 32; otherwise four overlapping quadrants cut on a 64-pixel grid
        (test_onesplit, refield 64), each run alone, stitched back."""
        h, w = x.size(2), x.size(3)
        if not self.training and h % 8 == 0 and w % 8 == 0 and h > 31 and w > 31:
            return self.forward_unet(x)
        if self.training or h < 32 or w < 32:
            return _test_pad(self.forward_unet, x, modulo=16)
        return _test_onesplit(self.forward_unet, x, refield=64)


def _test_pad(model, L, modulo: int = 16):
    """KAIR utils_model.test_pad: replicate-pad bottom / right to multiples of `modulo`, crop back."""
    h, w = L.size()[-2:]
    pb = int(np.ceil(h / modulo) * modulo - h)
    pr = int(np.ceil(w / modulo) * modulo - w)
    E = model(torch.nn.functional.pad(L, (0, pr, 0, pb), mode="replicate"))
    return E[..., :h, :w]


def _test_onesplit(model, L, refield: int = 32, sf: int = 1):
    """KAIR utils_model.test_onesplit: four corner crops of ((side // 2) // refield + 1) * refield
    pixels per side, each through the model, the four quarters of the output taken from them."""
    h, w = L.size()[-2:]
    th = (h // 2 // refield + 1) * refield
    tw = (w // 2 // refield + 1) * refield
    top, bottom = slice(0, th), slice(h - th, h)
    left, right = slice(0, tw), slice(w - tw, w)
    Es = [model(L[..., top, left]), model(L[..., top, right]), model(L[..., bottom, left]),
          model(L[..., bottom, right])]
    b, c = Es[0].size()[:2]
    E = torch.zeros(b, c, sf * h, sf * w, dtype=L.dtype, device=L.device)
    h2, w2 = h // 2 * sf, w // 2 * sf
    E[..., :h2, :w2] = Es[0][..., :h2, :w2]
    E[..., :h2, w2:w * sf] = Es[1][..., :h2, (-w + w // 2) * sf:]
    E[..., h2:h * sf, :w2] = Es[2][..., (-h + h // 2) * sf:, :w2]
    E[..., h2:h * sf, w2:w * sf] = Es[3][..., (-h + h // 2) * sf:, (-w + w // 2) * sf:]
    return E


def drunet_flops_per_pixel(nc=(64, 128, 256, 512), nb: int = 4, c: int = 3) -> float:
    """2 x MACs per input pixel of the DRUNet forward (level k runs on 4^-k of the pixels)."""
    macs = 9 * (c + 1) * nc[0] + 9 * nc[0] * c                        # head + tail
    for k, n in enumerate(nc):
        r = 4.0 ** -k
        blocks = 2 * nb if k < len(nc) - 1 else nb                      # down + up resblocks (body: nb)
        macs += r * blocks * 2 * 9 * n * n
        if k + 1 < len(nc):
            macs += (r / 4) * 4 * n * nc[k + 1] * 2                     # 2x2 down conv + 2x2 up transposed conv
    return 2.0 * macs


class DenoiserPrior:
    """prior_grad(x) = alpha * (denoiser.forward(x, s1) - x) / s2   (sampling_images.py:156-157)."""

    def __init__(self, denoiser, s1: float, alpha: torch.Tensor, s2: torch.Tensor):
        self.denoiser, self.s1, self.alpha, self.s2 = denoiser, s1, alpha, s2

    def __call__(self, x):
        return self.alpha * (self.denoiser.forward(x, self.s1) - x) / self.s2


def dncnn_flops_per_pixel(depth: int = 20, nf: int = 64, c: int = 3) -> float:
    """2 x MACs per output pixel of the DnCNN forward (1.334 MFLOP/pixel)."""
    macs = 9 * (c * nf + (depth - 2) * nf * nf + nf * c)
    return 2.0 * macs


__all__ = ["TVDenoiser", "DnCNN", "DRUNet", "DenoiserPrior", "dncnn_flops_per_pixel", "drunet_flops_per_pixel", "np"]
