"""oracle/psgla_oracle.py -- TEST INFRASTRUCTURE ONLY (the parity checker).

CPU (torch fp32, eager, op-for-op) restatement of the reference's hot path.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / CPU baseline: the product
package never imports it.

What it restates (all citations into /root/reference):

* ``psgla``   -- restoration_algorithms.py:163-285 (loop body :231-271)
* ``pnpula``  -- restoration_algorithms.py:38-160  (loop body :103-144)
* ``inpainting_problem`` / ``deblurring_problem`` -- the data-fidelity closures,
  observations and initialisations built by sampling_images.py:283-341
* ``TVDenoiser`` -- deepinv 0.2.1 ``deepinv.models.TVDenoiser`` (environment.yml:311;
  constructed sampling_images.py:138, called restoration_algorithms.py:238).
  deepinv is NOT vendored in /root/reference and not installed here: this is a
  restatement of the published 0.2.1 algorithm (Chambolle-Pock primal-dual,
  tau=0.01, rho=1.99, sigma=1/(8 tau), tol=1e-5, warm start in x2/u2).  Its
  arithmetic is "parity unpinned" by any reference fixture.
* the Gaussian noise ``torch.randn`` (restoration_algorithms.py:232, :104) is the
  injected "psgla noise v2" stream from oracle/noise.c (see its header): the
  golden fixtures were produced by the reference's own ``psgla``/``pnpula`` with
  ``torch.randn`` patched to return that stream (tests/golden/make_golden.py).

Pinning: tests/test_oracle_golden.py checks every function here against the
golden fixtures in tests/golden/ (bit-exact).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    """Load (building on first use if needed) oracle/liboracle_noise.so."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle_noise.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        lib = ctypes.CDLL(path)
        lib.oracle_normal_fill_rows.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        lib.oracle_philox4x32_10.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        lib.oracle_radius_table.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        lib.oracle_angle_table.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_uint32]
        _LIB = lib
    return _LIB


NOISE_TAG_LANGEVIN = 0


def normal(shape, seed: int, chain: int, step: int, tag: int = NOISE_TAG_LANGEVIN) -> torch.Tensor:
    """One Langevin step's N(0,1) draw for one chain (replaces torch.randn at
    restoration_algorithms.py:232 / :104): "psgla noise v2" over ``shape`` (the
    chain's (1,C,H,W) image) taken as rows of its last dimension -- element
    (row, col) is output col & 3 of quad row * ceil(W/4) + col // 4 (oracle/noise.c)."""
    n = int(np.prod(shape))
    W = int(shape[-1]) if len(shape) else 1
    out = np.empty(n, dtype=np.float32)
    if n:
        _lib().oracle_normal_fill_rows(out.ctypes.data, n // W, W, seed & ((1 << 64) - 1), chain, step, tag)
    return torch.from_numpy(out).reshape(shape)


def philox4x32_10(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    _lib().oracle_philox4x32_10(c, k, o)
    return list(o)


def radius_table(k_begin: int, count: int) -> np.ndarray:
    out = np.empty(count, dtype=np.float32)
    _lib().oracle_radius_table(out.ctypes.data, k_begin, count)
    return out


def angle_table(k_begin: int, count: int):
    c = np.empty(count, dtype=np.float32)
    s = np.empty(count, dtype=np.float32)
    _lib().oracle_angle_table(c.ctypes.data, s.ctypes.data, k_begin, count)
    return c, s


def sqrt_rn(t: torch.Tensor) -> torch.Tensor:
    """IEEE correctly rounded fp32 square root.  The reference executes on CUDA
    (sampling_images.py:109), where torch.sqrt(float32) is correctly rounded; torch's CPU
    AVX-512 float sqrt is not (about 0.5 % of values differ by one ulp), so the checker takes
    the float64 root and rounds it once to float32 -- the correctly rounded result."""
    if t.dtype != torch.float32:
        return torch.sqrt(t)
    return torch.sqrt(t.double()).float()


# --------------------------------------------------------------------------------------
# deepinv 0.2.1 TVDenoiser (restated; see module docstring)
# --------------------------------------------------------------------------------------
class TVDenoiser:
    """Isotropic TV proximal operator by primal-dual iterations with warm start.

    State ``x2`` (primal, (B,C,H,W)) and ``u2`` (dual, (B,C,H,W,2)) persist across
    calls; the first call (or a call with a new shape) restarts from x2=y, u2=0.
    """

    def __init__(self, n_it_max: int = 1000, tau: float = 0.01, rho: float = 1.99,
                 tol: float = 1e-5, verbose: bool = False):
        self.n_it_max = n_it_max
        self.tau = tau
        self.rho = rho
        self.crit = tol
        self.sigma = 1 / tau / 8
        self.restart = True
        self.x2 = None
        self.u2 = None
        self.verbose = verbose
        self.last_n_it = None          # inner iterations run by the last call (for tests)

    @staticmethod
    def nabla(x):
        """Forward differences, zero on the last row / column."""
        b, c, h, w = x.shape
        g = torch.zeros((b, c, h, w, 2), dtype=x.dtype)
        g[:, :, :-1, :, 0] = g[:, :, :-1, :, 0] - x[:, :, :-1]
        g[:, :, :-1, :, 0] = g[:, :, :-1, :, 0] + x[:, :, 1:]
        g[:, :, :, :-1, 1] = g[:, :, :, :-1, 1] - x[..., :-1]
        g[:, :, :, :-1, 1] = g[:, :, :, :-1, 1] + x[..., 1:]
        return g

    @staticmethod
    def nabla_adjoint(g):
        """Exact adjoint of :meth:`nabla` (negative divergence)."""
        b, c, h, w = g.shape[:-1]
        d = torch.zeros((b, c, h, w), dtype=g.dtype)
        d[:, :, :-1] = d[:, :, :-1] - g[:, :, :-1, :, 0]
        d[:, :, 1:] = d[:, :, 1:] + g[:, :, :-1, :, 0]
        d[..., :-1] = d[..., :-1] - g[..., :-1, 1]
        d[..., 1:] = d[..., 1:] + g[..., :-1, 1]
        return d

    def prox_tau_fx(self, x, y):
        return (x + self.tau * y) / (1 + self.tau)

    @staticmethod
    def prox_sigma_g_conj(u, lambda2):
        one = torch.tensor([1], dtype=u.dtype)
        return u / torch.maximum(sqrt_rn(torch.sum(u ** 2, axis=-1)) / lambda2, one).unsqueeze(-1)

    def forward(self, y, ths=None):
        if self.restart or self.x2 is None or self.x2.shape != y.shape:
            self.x2 = y.clone()
            self.u2 = torch.zeros((*y.shape, 2), dtype=y.dtype)
            self.restart = False
        lambd = ths
        it_done = 0
        for it in range(self.n_it_max):
            x_prev = self.x2.clone()
            x = self.prox_tau_fx(self.x2 - self.tau * self.nabla_adjoint(self.u2), y)
            u = self.prox_sigma_g_conj(self.u2 + self.sigma * self.nabla(2 * x - self.x2), lambd)
            self.x2 = self.x2 + self.rho * (x - self.x2)
            self.u2 = self.u2 + self.rho * (u - self.u2)
            it_done = it + 1
            rel_err = torch.linalg.norm(x_prev.flatten() - self.x2.flatten()) / \
                torch.linalg.norm(self.x2.flatten() + 1e-12)
            if it > 1 and rel_err < self.crit:
                break
        self.last_n_it = it_done
        return self.x2


class ClampDenoiser:
    """Cheap deterministic denoiser used by the fixtures: D(x, s) = clamp(x, 0, 1)."""

    def forward(self, x, sigma):
        return torch.clamp(x, 0.0, 1.0)


class TinyConvDenoiser:
    """Tiny residual 3x3 conv denoiser with fixed weights (pins the alpha != 1 relaxation)."""

    def __init__(self, weight: torch.Tensor, bias: torch.Tensor):
        self.weight = weight
        self.bias = bias

    def forward(self, x, sigma):
        return x - torch.nn.functional.conv2d(x, self.weight, self.bias, padding=1)


# --------------------------------------------------------------------------------------
# data-fidelity closures (sampling_images.py:283-341), restated
# --------------------------------------------------------------------------------------
def inpainting_problem(im_t: torch.Tensor, seed_ip: int = 0, prop: float = 0.5, sigma: float = 1.0):
    """Random-pixel inpainting: returns (data_grad, y_t, init, mask_2d).

    Same generator call sequence as sampling_images.py:285-302: one Generator
    seeded with seed_ip draws the (H,W) mask then the observation noise.
    """
    sigma1 = sigma / 255.0
    sigma2t = torch.tensor(sigma1 ** 2, dtype=torch.float32)
    gen = torch.Generator()
    gen.manual_seed(seed_ip)
    m = torch.rand((im_t.shape[2], im_t.shape[3]), generator=gen)
    mask_2d = 1 * (m > prop)
    mask = torch.ones(3)[None, :, None, None] * mask_2d[None, None, :, :]
    neg_mask = 1 - mask
    y_t = mask * im_t + torch.normal(torch.zeros(*im_t.size()), std=sigma1 * torch.ones(*im_t.size()),
                                     generator=gen)

    def data_grad(x):
        return -mask * (x - y_t) / sigma2t

    init = mask * y_t + neg_mask * 0.5 * torch.ones(y_t.shape)
    return data_grad, y_t, init, mask_2d


def blur_kernel(l: int = 4, blur_type: str = "uniform", si: float = 1.0) -> np.ndarray:
    """(2l+1)x(2l+1) blur kernel h_ = h^T h as built at sampling_images.py:306-313 (float64)."""
    if blur_type == "uniform":
        h = np.ones((1, 2 * l + 1))
    elif blur_type == "gaussian":
        h = np.array([[np.exp(-i ** 2 / (2 * si ** 2)) for i in range(-l, l + 1)]])
    else:
        raise ValueError(blur_type)
    h = h / np.sum(h)
    return np.dot(h.T, h)


def blur_operators(l: int = 4, blur_type: str = "uniform", si: float = 1.0, channels: int = 3):
    h_ = blur_kernel(l, blur_type, si)
    hconv = torch.from_numpy(np.copy(np.flip(h_))).type(torch.float32)
    hcorr = torch.from_numpy(h_).type(torch.float32)
    ones = torch.ones(channels, hconv.shape[0], hconv.shape[1])
    hconv = hconv.unsqueeze(0)[None] * ones[:, None]
    hcorr = hcorr.unsqueeze(0)[None] * ones[:, None]

    def A(x):
        return torch.nn.functional.conv2d(torch.nn.functional.pad(x, [l, l, l, l], mode="circular"),
                                          hconv, groups=x.size(1), padding=0)

    def AT(x):
        return torch.nn.functional.conv2d(torch.nn.functional.pad(x, [l, l, l, l], mode="circular"),
                                          hcorr, groups=x.size(1), padding=0)
    return A, AT


def blur_grad_tap_order(x: np.ndarray, y: np.ndarray, hconv: np.ndarray, hcorr: np.ndarray, l: int,
                        sigma2: float) -> np.ndarray:
    """-AT(A x - y) / sigma2 of ``blur_operators`` (sampling_images.py:329-338) with every output's
    (2l+1)^2-term sums taken in (row, column) tap order, one fp32 rounding per product and per sum --
    the order the HIP stencil's exact mode uses.  torch's CPU conv2d order is unspecified, so the
    reference closure itself is only matched to a tolerance; this restatement pins the kernel bit for bit.
    x, y: float32 (..., H, W); taps float32 (2l+1, 2l+1)."""
    K = 2 * l + 1
    hconv = np.asarray(hconv, np.float32)
    hcorr = np.asarray(hcorr, np.float32)

    def corr(v, h):
        acc = np.zeros_like(v)
        for u in range(K):
            for w in range(K):
                # conv2d(pad(v, l, circular), h)[i, j] = sum_{u,w} h[u, w] v[(i + u - l) % H, (j + w - l) % W]
                acc = acc + h[u, w] * np.roll(v, shift=(l - u, l - w), axis=(-2, -1))
        return acc

    r = corr(np.asarray(x, np.float32), hconv) - np.asarray(y, np.float32)
    return (-corr(r, hcorr)) / np.float32(sigma2)


def deblurring_problem(im_t: torch.Tensor, seed_ip: int = 0, l: int = 4, blur_type: str = "uniform",
                       si: float = 1.0, sigma: float = 1.0):
    """Circular (2l+1)^2 deblurring: returns (data_grad, y_t, init)."""
    sigma1 = sigma / 255.0
    sigma2t = torch.tensor(sigma1 ** 2, dtype=torch.float32)
    A, AT = blur_operators(l, blur_type, si, im_t.shape[1])
    gen = torch.Generator()
    gen.manual_seed(seed_ip)
    y_t = A(im_t) + torch.normal(torch.zeros(*im_t.size()), std=sigma1 * torch.ones(*im_t.size()),
                                 generator=gen)

    def data_grad(x):
        return -AT(A(x) - y_t) / sigma2t

    return data_grad, y_t, y_t


# --------------------------------------------------------------------------------------
# the two Langevin samplers (restoration_algorithms.py:38-160, :163-285), restated
# --------------------------------------------------------------------------------------
def _block_update(i_mmse, xmmse, xmmse2, X):
    xmmse = i_mmse / (i_mmse + 1) * xmmse + 1 / (i_mmse + 1) * X
    xmmse2 = i_mmse / (i_mmse + 1) * xmmse2 + 1 / (i_mmse + 1) * X ** 2
    return xmmse, xmmse2


def psgla(init, data_grad, denoiser, alpha, lambd, sig_float=0.0055, delta=4e-5, n_iter=5000,
          n_inter=1000, n_inter_mmse=1000, seed=None, chain: int = 0):
    """PSGLA chain on CPU; returns (Xlist, Xlist_mmse, Xlist_mmse2) like the reference."""
    dtype = torch.float32
    shape = init.shape
    X = init.clone().detach()
    xmmse = torch.zeros(shape, dtype=dtype)
    xmmse2 = torch.zeros(shape, dtype=dtype)
    delta_t = torch.tensor(delta).to(torch.float32)
    sig = torch.tensor(sig_float).to(torch.float32)
    if seed is None:
        raise UnboundLocalError("local variable 'gen' referenced before assignment")
    if n_inter_mmse is None:
        n_inter_mmse = np.copy(n_inter)
    Xlist, Xlist_mmse, Xlist_mmse2 = [], [], []
    i_mmse = 0
    K = int(n_iter / 10)
    noise_ratio = torch.tensor(np.sqrt(2)).to(torch.float32)
    with torch.no_grad():
        for i in range(n_iter):
            Z = normal(shape, seed, chain, i)
            g = data_grad(X)
            Y = X + (delta_t / lambd) * g + noise_ratio * sig * Z
            X = (1 - alpha) * Y + alpha * denoiser.forward(Y, sig)
            if i % n_inter == 0:
                Xlist.append(torch.squeeze(X))
            i % K  # noqa: B018 -- the reference evaluates i % K every step (ZeroDivisionError if n_iter < 10)
            xmmse, xmmse2 = _block_update(i_mmse, xmmse, xmmse2, X)
            if i_mmse <= n_inter_mmse - 1:
                i_mmse += 1
            else:
                Xlist_mmse.append(torch.squeeze(xmmse))
                Xlist_mmse2.append(torch.squeeze(xmmse2))
                xmmse = torch.zeros(shape, dtype=dtype)
                xmmse2 = torch.zeros(shape, dtype=dtype)
                i_mmse = 0
    return Xlist, Xlist_mmse, Xlist_mmse2


def pnpula(init, data_grad, prior_grad, delta, lambd, n_iter=5000, n_inter=1000, n_inter_mmse=1000,
           seed=None, c_min=-1, c_max=2, chain: int = 0):
    """PnP-ULA chain on CPU; returns (Xlist, Xlist_mmse, Xlist_mmse2) like the reference."""
    dtype = torch.float32
    shape = init.shape
    X = init.clone().detach()
    one = torch.ones(shape, dtype=dtype)
    xmmse = torch.zeros(shape, dtype=dtype)
    xmmse2 = torch.zeros(shape, dtype=dtype)
    brw = sqrt_rn(2 * delta)
    if seed is None:
        raise UnboundLocalError("local variable 'gen' referenced before assignment")
    if n_inter_mmse is None:
        n_inter_mmse = np.copy(n_inter)
    Xlist, Xlist_mmse, Xlist_mmse2 = [], [], []
    i_mmse = 0
    K = int(n_iter / 10)
    with torch.no_grad():
        for i in range(n_iter):
            Z = normal(shape, seed, chain, i)
            gp = prior_grad(X)
            gd = data_grad(X)
            out = torch.where(X > c_min, X, c_min * one)
            proj = torch.where(out < c_max, out, c_max * one)
            grad_pi = gp - (X - proj) / lambd + gd
            X = X + delta * grad_pi + brw * Z
            if i % n_inter == 0:
                Xlist.append(torch.squeeze(X))
            i % K  # noqa: B018
            xmmse, xmmse2 = _block_update(i_mmse, xmmse, xmmse2, X)
            if i_mmse <= n_inter_mmse - 1:
                i_mmse += 1
            else:
                Xlist_mmse.append(torch.squeeze(xmmse))
                Xlist_mmse2.append(torch.squeeze(xmmse2))
                xmmse = torch.zeros(shape, dtype=dtype)
                xmmse2 = torch.zeros(shape, dtype=dtype)
                i_mmse = 0
    return Xlist, Xlist_mmse, Xlist_mmse2


def mmse_of_blocks(blocks):
    """Final MMSE = mean of the block means (sampling_images.py:412, :428)."""
    return np.mean(np.array([b.numpy() for b in blocks]), axis=0)


def psgla_params_tv(s_pix: float = 10.0, lambd: float = 10.0):
    """PSGLA+TV constants of sampling_images.py:180-198 (flags not typed)."""
    s = s_pix / 255.0
    return dict(s=s, lambd=lambd, delta=s ** 2)


def psgla_coefficients(delta_float: float, lambd: float, s: float):
    """(c1 = delta/lambd, c2 = sqrt(2) * s) exactly as the fp32 0-d tensor ops of
    restoration_algorithms.py:203-205, :228, :236 evaluate them."""
    d = torch.tensor(delta_float).to(torch.float32)
    lam = torch.tensor(lambd, dtype=torch.float32)
    c1 = (d / lam).item()
    c2 = (torch.tensor(np.sqrt(2)).to(torch.float32) * torch.tensor(s).to(torch.float32)).item()
    return c1, c2


__all__ = [
    "normal", "philox4x32_10", "radius_table", "angle_table", "TVDenoiser", "ClampDenoiser",
    "TinyConvDenoiser", "inpainting_problem", "blur_kernel", "blur_operators", "blur_grad_tap_order", "deblurring_problem",
    "psgla", "pnpula", "mmse_of_blocks", "psgla_params_tv", "psgla_coefficients", "math",
]
