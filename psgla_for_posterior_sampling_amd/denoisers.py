"""Denoisers with deepinv 0.2.1's call protocol ``denoiser.forward(x, sigma)``.

* :class:`TVDenoiser` -- deepinv.models.TVDenoiser (constructed at sampling_images.py:138,
  called at restoration_algorithms.py:238) on the HIP TV-prox kernel: same constructor
  arguments, same warm-start state (``x2``, ``u2``, ``restart``), same early stop.
* :class:`DnCNN` -- deepinv.models.DnCNN architecture (sampling_images.py:130): 20 conv3x3
  layers, 64 features, ReLU, residual output; parameter names ``in_conv`` / ``conv_list.i`` /
  ``out_conv`` so a deepinv ``state_dict`` loads unchanged.  Runs on PyTorch-ROCm (MIOpen),
  as the north star prescribes for the DNN forward.
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

    def forward(self, y, ths=None):
        if ths is None:
            raise TypeError("TVDenoiser.forward needs the threshold `ths` (the reference passes sigma)")
        y = y.contiguous()
        fresh = self.needs_restart(y.shape)
        k = self.constants()
        if self._work is None or self._work.norms.shape[1] != max(k.n_it, 1) or self._work.norms.device != y.device:
            self._work = K.TvWorkspace(1, k.n_it, y.device)
        x2, u2 = K.tv_prox(y, float(ths), k, None if fresh else self.x2, None if fresh else self.u2,
                           fresh=fresh, exact=self.exact, work=self._work)
        self.x2, self.u2 = x2, u2
        self.restart = False
        return x2


class DnCNN(torch.nn.Module):
    """deepinv DnCNN(in_channels=3, out_channels=3, depth=20, nf=64, bias=True), residual."""

    def __init__(self, in_channels: int = 3, out_channels: int = 3, depth: int = 20, bias: bool = True,
                 nf: int = 64, pretrained: str | None = None, device="cpu"):
        super().__init__()
        self.depth = depth
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

    def forward(self, x, sigma=None):
        x1 = self.nl_list[0](self.in_conv(x))
        for i in range(self.depth - 2):
            x1 = self.nl_list[i + 1](self.conv_list[i](x1))
        return self.out_conv(x1) + x


def dncnn_flops_per_pixel(depth: int = 20, nf: int = 64, c: int = 3) -> float:
    """2 x MACs per output pixel of the DnCNN forward (1.334 MFLOP/pixel)."""
    macs = 9 * (c * nf + (depth - 2) * nf * nf + nf * c)
    return 2.0 * macs


__all__ = ["TVDenoiser", "DnCNN", "dncnn_flops_per_pixel", "np"]
