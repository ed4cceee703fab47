"""Torch-tensor wrappers over the C ABI (include/psgla_hip.h).

Every wrapper launches on the *current* torch stream, so the ops compose with PyTorch
work (the DnCNN/DRUNet forward) and are captured by ``torch.cuda.graph``.  Inputs must
be contiguous fp32 CUDA tensors; nothing here falls back to PyTorch or the CPU.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as N

NOISE_TAG_LANGEVIN = 0


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: torch.Tensor | None, dtype=torch.float32, name: str = "tensor") -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor, got device {t.device}")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t.data_ptr()


def _bce(x: torch.Tensor):
    if x.dim() < 2:
        raise ValueError("expected a (B, ...) tensor")
    B = x.shape[0]
    return B, x.numel() // B


def _row(x: torch.Tensor) -> int:
    """Row length of a chain's image for the noise (psgla noise v2: quads never straddle two rows)."""
    return int(x.shape[-1])


# ------------------------------------------------------------------------------------
# accumulation schedule (restoration_algorithms.py:240-271)
# ------------------------------------------------------------------------------------
def acc_coefficients(n_inter_mmse: int) -> np.ndarray:
    """(fp32(k/(k+1)), fp32(1/(k+1))) for k = 0..n_inter_mmse, exactly as the reference's
    Python-float scalars reach its fp32 tensor multiplications."""
    k = np.arange(int(n_inter_mmse) + 1, dtype=np.float64)
    return np.stack([np.float32(k / (k + 1)), np.float32(1.0 / (k + 1))], axis=1).astype(np.float32).ravel()


class Schedule:
    """Device-side schedule of one chain batch: step counter, block-mean coefficients,
    preallocated sample / block storage (the reference keeps these on the device too)."""

    def __init__(self, shape, n_iter: int, n_inter: int, n_inter_mmse: int, device,
                 store_samples: bool = True, store_blocks: bool = True, d_step: torch.Tensor | None = None):
        self.shape = tuple(shape)
        self.n_iter = int(n_iter)
        self.n_inter = int(n_inter)
        self.n_inter_mmse = int(n_inter_mmse)
        self.device = torch.device(device)
        per = self.n_inter_mmse + 1
        self.samples_cap = (self.n_iter + self.n_inter - 1) // self.n_inter if (store_samples and self.n_inter > 0) else 0
        self.blocks_cap = self.n_iter // per if store_blocks else 0
        self.coef = torch.from_numpy(acc_coefficients(self.n_inter_mmse)).to(self.device)
        self.samples = torch.empty((max(self.samples_cap, 0),) + self.shape, dtype=torch.float32, device=self.device) \
            if self.samples_cap > 0 else None
        self.blocks = torch.empty((self.blocks_cap,) + self.shape, dtype=torch.float32, device=self.device) \
            if self.blocks_cap > 0 else None
        self.blocks2 = torch.empty_like(self.blocks) if self.blocks is not None else None
        self.d_step = d_step if d_step is not None else torch.zeros(1, dtype=torch.int64, device=self.device)

    def struct(self, use_device_step: bool = True, step_offset: int = 0) -> N.PsglaSchedule:
        s = N.PsglaSchedule()
        s.d_step = self.d_step.data_ptr() if use_device_step else None
        s.step_offset = int(step_offset)
        s.n_inter = self.n_inter
        s.n_inter_mmse = self.n_inter_mmse
        s.acc_coef = self.coef.data_ptr()
        s.samples = self.samples.data_ptr() if self.samples is not None else None
        s.samples_cap = self.samples_cap
        s.blocks = self.blocks.data_ptr() if self.blocks is not None else None
        s.blocks2 = self.blocks2.data_ptr() if self.blocks2 is not None else None
        s.blocks_cap = self.blocks_cap
        return s

    def n_samples_done(self, steps_done: int) -> int:
        if self.n_inter <= 0:
            return 0
        return min(self.samples_cap, (steps_done + self.n_inter - 1) // self.n_inter)

    def n_blocks_done(self, steps_done: int) -> int:
        return min(self.blocks_cap, steps_done // (self.n_inter_mmse + 1))


# ------------------------------------------------------------------------------------
# generic building blocks
# ------------------------------------------------------------------------------------
def normal_fill(out: torch.Tensor, seed: int, chain0: int, step: int, tag: int = NOISE_TAG_LANGEVIN,
                d_step: torch.Tensor | None = None):
    B, E = _bce(out)
    N.check(N.lib().psgla_normal_fill(_ptr(out, name="out"), B, E, _row(out), seed & (2 ** 64 - 1), chain0,
                                      d_step.data_ptr() if d_step is not None else None, step, tag,
                                      _stream()), "psgla_normal_fill")
    return out


def langevin_update(X, g, c1: float, c2: float, seed: int, chain0: int, step: int, out=None,
                    d_step: torch.Tensor | None = None):
    if out is None:
        out = torch.empty_like(X)
    B, E = _bce(X)
    N.check(N.lib().psgla_langevin_update(_ptr(X, name="X"), _ptr(g, name="g"), _ptr(out, name="Y"), B, E,
                                          _row(X), c1, c2, seed & (2 ** 64 - 1), chain0,
                                          d_step.data_ptr() if d_step is not None else None, step,
                                          _stream()), "psgla_langevin_update")
    return out


def relax_accumulate(Y, D, X_out, alpha: float, mean, sq, sched: Schedule, step: int,
                     use_device_step: bool = False):
    B, E = _bce(Y)
    s = sched.struct(use_device_step, step)
    N.check(N.lib().psgla_relax_accumulate(_ptr(Y, name="Y"), _ptr(D, name="D"), _ptr(X_out, name="X"),
                                           alpha, int(alpha == 1.0), _ptr(mean, name="mean"), _ptr(sq, name="sq"),
                                           B, E, ctypes.byref(s), _stream()), "psgla_relax_accumulate")
    return X_out


def relax_langevin_inpaint(Y, D, alpha: float, y, mask_u8, sigma2: float, c1: float, c2: float, seed: int,
                           chain0: int, mean, sq, sched: Schedule, step: int, Y_next, X_out=None,
                           use_device_step: bool = False):
    """Epilogue of step `step` + prologue of step `step + 1` for the inpainting fidelity (one pass):
    X = (1-alpha) Y + alpha D, accumulators, Y_next = (X + c1 g(X)) + c2 Z_{step+1}."""
    B, C, H, W = D.shape
    alpha1 = float(alpha) == 1.0
    y_cs = 0 if y.shape[0] == 1 else C * H * W
    m_cs = 0 if (mask_u8.dim() == 2 or mask_u8.shape[0] == 1) else H * W
    s = sched.struct(use_device_step, step)
    N.check(N.lib().psgla_relax_langevin_inpaint(
        None if alpha1 else _ptr(Y, name="Y"), _ptr(D, name="D"), _ptr(X_out, name="X") if X_out is not None else None,
        float(alpha), int(alpha1), _ptr(y, name="y"), y_cs, _ptr(mask_u8, torch.uint8, "mask"), m_cs,
        _ptr(Y_next, name="Y_next"), _ptr(mean, name="mean"), _ptr(sq, name="sq"), B, C, H, W, float(sigma2),
        float(c1), float(c2), seed & (2 ** 64 - 1), int(chain0), ctypes.byref(s), _stream()),
        "psgla_relax_langevin_inpaint")
    return Y_next


def pnpula_update(X, gp, gd, X_out, delta: float, lambd: float, brw: float, c_min: float, c_max: float,
                  mean, sq, sched: Schedule, step: int, seed: int, chain0: int, use_device_step: bool = False):
    B, E = _bce(X)
    s = sched.struct(use_device_step, step)
    N.check(N.lib().pnpula_update(_ptr(X, name="X"), _ptr(gp, name="gp"), _ptr(gd, name="gd"),
                                  _ptr(X_out, name="Xout"), delta, lambd, brw, c_min, c_max,
                                  _ptr(mean, name="mean"), _ptr(sq, name="sq"), B, E, _row(X), seed & (2 ** 64 - 1),
                                  chain0, ctypes.byref(s), _stream()), "pnpula_update")
    return X_out


def pnpula_prior_update(X, D, alpha: float, s2: float, X_out, delta: float, lambd: float, brw: float, c_min: float,
                        c_max: float, mean, sq, sched: Schedule, step: int, seed: int, chain0: int, *, gd=None, y=None,
                        mask_u8=None, sigma2: float = 1.0, use_device_step: bool = False):
    """PnP-ULA step with the DNN prior fused (V-ULA): gp = (alpha (D - X)) / s2, the inpainting data term
    (y, mask_u8, sigma2) or a given gd, the update, noise and accumulators in one HIP pass."""
    B, C, H, W = X.shape
    s = sched.struct(use_device_step, step)
    y_cs = 0 if (y is None or y.shape[0] == 1) else C * H * W
    m_cs = 0 if (mask_u8 is None or mask_u8.dim() == 2 or mask_u8.shape[0] == 1) else H * W
    N.check(N.lib().pnpula_prior_update(
        _ptr(X, name="X"), _ptr(D, name="D"), float(alpha), float(s2), _ptr(gd, name="gd") if gd is not None else None,
        _ptr(y, name="y") if y is not None else None, y_cs,
        _ptr(mask_u8, torch.uint8, "mask") if mask_u8 is not None else None, m_cs, float(sigma2),
        _ptr(X_out, name="Xout"), float(delta), float(lambd), float(brw), float(c_min), float(c_max),
        _ptr(mean, name="mean"), _ptr(sq, name="sq"), B, C, H, W, seed & (2 ** 64 - 1), int(chain0), ctypes.byref(s),
        _stream()), "pnpula_prior_update")
    return X_out


def bias_act_(y: torch.Tensor, bias: torch.Tensor, relu: bool = True) -> torch.Tensor:
    """In place y = relu(y + bias[c]) (or y + bias[c]) for an (N, C, H, W) conv output in NHWC
    (channels_last) or NCHW memory; the DnCNN layer epilogue (one HBM pass instead of two)."""
    N_, C, H, W = y.shape
    if y.is_contiguous(memory_format=torch.channels_last) and C % 4 == 0:
        hw = 0
        ptr = y.data_ptr()
        if y.dtype != torch.float32 or not y.is_cuda:
            raise TypeError("bias_act_: y must be a CUDA float32 tensor")
    else:
        hw = H * W
        ptr = _ptr(y, name="y")
    b = bias.contiguous()
    N.check(N.lib().psgla_bias_act(ptr, _ptr(b, name="bias"), y.numel(), C, hw, 1 if relu else 0, _stream()),
            "psgla_bias_act")
    return y


def inpaint_grad(X, y, mask_u8, sigma2: float, out=None):
    """g = ((-m)(X - y)) / sigma2 with mask (H,W) or (B,H,W) uint8 and y (B|1,C,H,W)."""
    B, C, H, W = X.shape
    if out is None:
        out = torch.empty_like(X)
    y_cs = 0 if y.shape[0] == 1 else C * H * W
    m_cs = 0 if (mask_u8.dim() == 2 or mask_u8.shape[0] == 1) else H * W
    N.check(N.lib().psgla_inpaint_grad(_ptr(X, name="X"), _ptr(y, name="y"), y_cs,
                                       _ptr(mask_u8, torch.uint8, "mask"), m_cs, _ptr(out, name="g"), B, C, H, W,
                                       sigma2, _stream()), "psgla_inpaint_grad")
    return out


def _host_taps(h, l: int) -> np.ndarray:
    t = h.detach().cpu().numpy() if isinstance(h, torch.Tensor) else np.asarray(h)
    t = np.ascontiguousarray(t, dtype=np.float32)
    if t.shape != (2 * l + 1, 2 * l + 1):
        raise ValueError(f"blur taps must be ({2 * l + 1}, {2 * l + 1}), got {t.shape}")
    return t


def blur_grad(X, y, hconv, hcorr, l: int, sigma2: float, out=None, exact: bool = False):
    """g = -A^T(A X - y) / sigma2 (circular depthwise (2l+1)^2 stencils, sampling_images.py:329-338).
    hconv / hcorr: (2l+1, 2l+1) fp32 taps shared by every channel (host copies are passed)."""
    B, C, H, W = X.shape
    if out is None:
        out = torch.empty_like(X)
    y_cs = 0 if y.shape[0] == 1 else C * H * W
    hc, hr = _host_taps(hconv, l), _host_taps(hcorr, l)
    N.check(N.lib().psgla_blur_grad(_ptr(X, name="X"), _ptr(y, name="y"), y_cs, hc.ctypes.data,
                                    hr.ctypes.data, int(l), _ptr(out, name="g"), None, B, C, H, W,
                                    sigma2, 0.0, 0.0, 0, 0, None, 0, int(exact), _stream()), "psgla_blur_grad")
    return out


def blur_set_separable(enable: bool) -> None:
    """Fast-mode rank-1 taps take the separable row / column passes (default) or, with False, the
    2-D stencil (process-wide; A/B and tests)."""
    N.check(N.lib().psgla_blur_set_separable(int(bool(enable))), "psgla_blur_set_separable")


def blur_langevin(X, y, hconv, hcorr, l: int, sigma2: float, c1: float, c2: float, seed: int, chain0: int,
                  step: int, out=None, exact: bool = False, d_step: torch.Tensor | None = None):
    """Y = (X + c1 g(X)) + c2 Z with the deblurring g fused (restoration_algorithms.py:232-236)."""
    B, C, H, W = X.shape
    if out is None:
        out = torch.empty_like(X)
    y_cs = 0 if y.shape[0] == 1 else C * H * W
    hc, hr = _host_taps(hconv, l), _host_taps(hcorr, l)
    N.check(N.lib().psgla_blur_grad(_ptr(X, name="X"), _ptr(y, name="y"), y_cs, hc.ctypes.data,
                                    hr.ctypes.data, int(l), None, _ptr(out, name="Y"), B, C, H, W,
                                    sigma2, c1, c2, seed & (2 ** 64 - 1), chain0,
                                    d_step.data_ptr() if d_step is not None else None, step, int(exact),
                                    _stream()), "psgla_blur_grad")
    return out


def advance_step(d_step: torch.Tensor):
    N.check(N.lib().psgla_advance_step(_ptr(d_step, torch.int64, "d_step"), _stream()), "psgla_advance_step")


# ------------------------------------------------------------------------------------
# TV prox (deepinv 0.2.1 TVDenoiser.forward semantics)
# ------------------------------------------------------------------------------------
class TvConstants:
    """fp32 constants of the TV prox exactly as deepinv's Python scalars reach fp32 ops."""

    def __init__(self, tau: float = 0.01, rho: float = 1.99, tol: float = 1e-5, n_it_max: int = 10):
        self.tau = float(np.float32(tau))
        self.one_plus_tau = float(np.float32(1 + tau))
        self.sigma_tv = float(np.float32(1 / tau / 8))
        self.rho = float(np.float32(rho))
        self.tol = float(tol)
        self.n_it = int(n_it_max)


def _tv_prox_launch(y, ths, k: TvConstants, n_it: int, x2_in, u2_in, fresh: bool, exact: bool, x2_out, u2_out,
                    work, per_chain: bool, it0: int, last: bool, stopped):
    B, C, H, W = y.shape
    d = N.PsglaTvProx()
    d.B, d.C, d.H, d.W = B, C, H, W
    d.y = _ptr(y, name="y")
    d.x2_in = _ptr(x2_in, name="x2_in") if not fresh else None
    d.u2_in = _ptr(u2_in, name="u2_in") if not fresh else None
    d.x2_out = _ptr(x2_out, name="x2_out")
    d.u2_out = _ptr(u2_out, name="u2_out")
    d.tau, d.one_plus_tau, d.sigma_tv, d.rho = k.tau, k.one_plus_tau, k.sigma_tv, k.rho
    d.ths = float(np.float32(ths))
    d.tol = k.tol
    d.n_tv = n_it
    d.exact = int(bool(exact))
    d.fresh = int(bool(fresh))
    d.norms = work.norms.data_ptr()
    d.arrive = work.arrive.data_ptr()
    d.per_chain = int(bool(per_chain))
    d.it0 = int(it0)
    d.last_chunk = int(bool(last))
    d.stopped = stopped.data_ptr() if stopped is not None else None
    N.check(N.lib().psgla_tv_prox(ctypes.byref(d), _stream()), "psgla_tv_prox")


def tv_prox(y: torch.Tensor, ths: float, k: TvConstants, x2_in=None, u2_in=None, fresh: bool = True,
            exact: bool = False, x2_out=None, u2_out=None, work=None, per_chain: bool = False):
    """One TVDenoiser.forward on the GPU; returns (x2_out, u2_out).

    per_chain: deepinv's early stop on each chain of the batch (B independent reference runs) instead
    of on the whole tensor.  n_it_max above N.TV_MAX_FUSED_IT runs as chunks of at most that many
    inner iterations (psgla_tv_prox's it0 / last_chunk / stopped): after each chunk but the last the
    host reads which groups stopped inside it and keeps their result (one host sync per chunk)."""
    B, C, H, W = y.shape
    G = B if per_chain else 1
    if x2_out is None:
        x2_out = torch.empty_like(y)
    if u2_out is None:
        u2_out = torch.empty(y.shape + (2,), dtype=torch.float32, device=y.device)
    n = k.n_it
    cmax = N.TV_MAX_FUSED_IT
    if work is None or work.norms.shape[0] < G or work.norms.shape[1] < min(max(n, 1), cmax):
        work = TvWorkspace(G, min(max(n, 1), cmax), y.device)
    if n <= cmax:
        _tv_prox_launch(y, ths, k, n, x2_in, u2_in, fresh, exact, x2_out, u2_out, work, per_chain, 0, True, None)
        return x2_out, u2_out
    # chunked: ping-pong between two scratch pairs; a group's result is final at its stop
    bufs = [(torch.empty_like(y), torch.empty_like(u2_out)) for _ in range(2)]
    stopped = torch.zeros(G, dtype=torch.int32, device=y.device)
    done = np.zeros(G, dtype=bool)
    cur_x2, cur_u2, cur_fresh = x2_in, u2_in, fresh
    nch = (n + cmax - 1) // cmax
    rows = (lambda g: slice(g, g + 1)) if per_chain else (lambda g: slice(None))
    for c in range(nch):
        it0 = c * cmax
        last = c == nch - 1
        ox2, ou2 = bufs[c & 1]
        _tv_prox_launch(y, ths, k, min(cmax, n - it0), cur_x2, cur_u2, cur_fresh, exact, ox2, ou2, work, per_chain,
                        it0, last, None if last else stopped)
        cur_x2, cur_u2, cur_fresh = ox2, ou2, False
        if last:
            break
        st = stopped.cpu().numpy()
        for g in np.nonzero((st > 0) & ~done)[0]:
            x2_out[rows(g)].copy_(ox2[rows(g)])
            u2_out[rows(g)].copy_(ou2[rows(g)])
            done[g] = True
        if done.all():
            return x2_out, u2_out
    for g in np.nonzero(~done)[0]:
        x2_out[rows(g)].copy_(cur_x2[rows(g)])
        u2_out[rows(g)].copy_(cur_u2[rows(g)])
    return x2_out, u2_out


class TvWorkspace:
    """Zero-initialised early-stop workspace: norms[groups][n_it][2] (fp64) + arrival counter.  copies > 1:
    norms_all holds that many such arrays back to back (PsglaTvStep.norms_copies), `norms` is the first."""

    def __init__(self, groups: int, n_it: int, device, copies: int = 1):
        self.copies = max(int(copies), 1)
        self.norms_all = torch.zeros((self.copies * max(groups, 1), max(n_it, 1), 2), dtype=torch.float64,
                                     device=device)
        self.norms = self.norms_all[:max(groups, 1)]
        self.arrive = torch.zeros(4, dtype=torch.int32, device=device)
        self.fresh = torch.zeros(4, dtype=torch.int32, device=device)
        # parallel early-stop redo state (PsglaTvStep.redo, ABI 11): [0] pending, [1] grid barrier, [4 + g] stop counts
        self.redo = torch.zeros(4 + max(groups, 1), dtype=torch.int32, device=device)
