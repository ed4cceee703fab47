"""Drop-in ``psgla`` / ``pnpula`` (reference restoration_algorithms.py:163 and :38).

Same signatures, argument meaning, return value (three lists of squeezed device tensors:
samples every ``n_inter`` steps, block means of X and of X**2) and error behaviour
(ZeroDivisionError when ``n_iter < 10`` or ``n_inter == 0``; UnboundLocalError when
``seed is None``, because the reference only creates its generator for a given seed).

Dispatch:
* ``data_grad`` an :class:`InpaintingFidelity` and ``denoiser`` a :class:`TVDenoiser` ->
  the fused HIP step (one kernel launch per Langevin step, hipGraph-replayed): config 2.
* a typed data term (:class:`InpaintingFidelity` / :class:`BlurFidelity`) and a PyTorch
  denoiser (DnCNN, DRUNet, any ``torch.nn.Module``) -> :class:`engine.DenoiserChains`: per step
  the denoiser forward on PyTorch-ROCm, then one HIP pass (inpainting: relaxation, accumulators
  and the next step's Langevin update fused) or two (deblurring: relaxation + accumulators, stencil
  with the Langevin update fused); the step index lives on the device and, for this package's
  DnCNN / DRUNet, ``graph_steps`` steps are captured in one hipGraph and replayed: configs 3-4.
* anything else (opaque closures) -> the closures are called as given, and the rest of the
  step (Gaussian noise, Langevin update, relaxation, accumulators, sample storage) runs as HIP
  kernels; a ``BlurFidelity`` data term is fused with the Langevin update (one stencil kernel).
``pnpula`` with a :class:`~denoisers.DenoiserPrior` prior and a typed data term runs
:class:`engine.UlaChains` (hipGraph-replayed steps: config 5).
The Gaussian noise is the in-kernel "psgla noise v2" stream of (seed, chain) instead of
torch's generator (whose CUDA stream depends on the device's CU count); extra keyword
``chain0`` gives the global id of the first chain when a batch is sharded over GPUs.

Batches: ``init`` may be (B, C, H, W) -- B independent chains (chain ids chain0..chain0+B-1),
each behaving exactly like one reference run.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import hip_ops as K
from .denoisers import DenoiserPrior, DnCNN, DRUNet, TVDenoiser
from .engine import DenoiserChains, FusedTvChains, UlaChains
from .fidelity import BlurFidelity, InpaintingFidelity

DEFAULT_GRAPH_STEPS = int(os.environ.get("PSGLA_GRAPH_STEPS", "50"))


def _check_schedule(n_iter, n_inter, n_inter_mmse, seed):
    if seed is None:
        raise UnboundLocalError("local variable 'gen' referenced before assignment")
    if n_inter_mmse is None:
        n_inter_mmse = int(np.copy(n_inter))
    K_ = int(n_iter / 10)
    if n_iter > 0 and (K_ == 0 or n_inter == 0):
        raise ZeroDivisionError("integer division or modulo by zero")
    return int(n_inter), int(n_inter_mmse), K_


def _lists(sched: K.Schedule, steps_done: int):
    ns = sched.n_samples_done(steps_done)
    nb = sched.n_blocks_done(steps_done)
    Xlist = [torch.squeeze(sched.samples[k]) for k in range(ns)] if sched.samples is not None else []
    M = [torch.squeeze(sched.blocks[k]) for k in range(nb)] if sched.blocks is not None else []
    M2 = [torch.squeeze(sched.blocks2[k]) for k in range(nb)] if sched.blocks2 is not None else []
    return Xlist, M, M2


class _Snapshots:
    """``save_images_online`` (restoration_algorithms.py:246-253 + :273-283 for psgla, :124-127 +
    :146-158 for pnpula): after every step i with i % K == 0 (K = int(n_iter / 10)), x_i.png (and
    y_i.png for psgla) of chain 0 -- the reference runs one chain, ``X.numpy()[0]`` --, then
    ``torch.save`` of the dict {'Samples', 'Mmse', 'Mmse2', <run parameters>} with the lists as they
    stand after step i.  The list tensors are saved as copies: views would serialise the whole
    sample / block store they live in."""

    def __init__(self, path, name, extra):
        self.path, self.name, self.extra = path, name, extra

    @staticmethod
    def _png(fname, t):
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        a = np.transpose(t.detach().cpu().numpy()[0, :, :, :], (1, 2, 0))
        plt.imsave(fname, np.clip(a, 0, 1), cmap=None)

    def save(self, i, X, Y, lists):
        self._png(self.path + "/x_" + str(i) + ".png", X)
        if Y is not None:
            self._png(self.path + "/y_" + str(i) + ".png", Y)
        Xl, M, M2 = lists
        d = {"Samples": [t.clone() for t in Xl], "Mmse": [t.clone() for t in M], "Mmse2": [t.clone() for t in M2]}
        d.update(self.extra)
        torch.save(d, self.path + "/" + self.name + "_sampling.pth")


def _run_with_snapshots(run, n_iter: int, Kfreq: int, snap):
    """Run n_iter steps through ``run(n)`` and call ``snap(i)`` right after every step i with
    i % Kfreq == 0 (the reference's cadence, restoration_algorithms.py:246, :273)."""
    done = 0
    for i in range(0, n_iter, Kfreq):
        run(i + 1 - done)
        done = i + 1
        snap(i)
    run(n_iter - done)


def psgla(init, data_grad, denoiser, alpha, lambd, sig_float=0.0055, delta=4e-5, n_iter=5000, n_inter=1000,
          n_inter_mmse=1000, seed=None, device=None, path=None, save_images_online=False, name=None, *,
          chain0: int = 0, graph_steps: int | None = None, exact: bool | None = None):
    """Proximal Stochastic Gradient Langevin Algorithm (restoration_algorithms.py:163-285)."""
    if device is None:
        device = init.device
    if not init.is_cuda:
        raise ValueError("psgla runs on the GPU: init must be a CUDA (HIP) tensor")
    delta_float = delta
    sig_noised = sig_float
    print("delta = {}, sigma = {}".format(delta_float, sig_noised))
    path = "" if path is None else path
    name = "" if name is None else name
    n_inter, n_inter_mmse, Kfreq = _check_schedule(n_iter, n_inter, n_inter_mmse, seed)
    dev = init.device
    X0 = init.clone().detach().contiguous().float()
    shape = X0.shape if X0.dim() == 4 else (1,) + tuple(X0.shape)
    X0 = X0.reshape(shape)
    delta_t = torch.tensor(delta_float).to(torch.float32)
    lambd_t = torch.as_tensor(lambd).detach().cpu().to(torch.float32)
    c1 = float((delta_t / lambd_t).item())
    c2 = float((torch.tensor(np.sqrt(2)).to(torch.float32) * torch.tensor(sig_noised).to(torch.float32)).item())
    alpha_f = float(torch.as_tensor(alpha).detach().cpu().to(torch.float32).item())
    seed = int(seed)
    if graph_steps is None:
        graph_steps = DEFAULT_GRAPH_STEPS

    snaps = None
    if save_images_online:
        snaps = _Snapshots(path, name, {"n_iter": n_iter, "lambda": lambd, "delta": delta_t.to(dev)})

    fused = (isinstance(data_grad, InpaintingFidelity) and isinstance(denoiser, TVDenoiser)
             and denoiser.n_it_max <= K.N.TV_MAX_FUSED_IT)
    if fused:
        if exact is None:
            exact = denoiser.exact
        warm = not denoiser.needs_restart(shape)
        eng = FusedTvChains(X0, data_grad.y, data_grad.mask_u8, c1=c1, c2=c2, sigma2=data_grad.sigma2,
                            alpha=alpha_f, ths=float(np.float32(sig_noised)), tv=denoiser.constants(), seed=seed,
                            n_iter=n_iter, n_inter=n_inter, n_inter_mmse=n_inter_mmse, chain0=chain0,
                            exact=exact, tv_x2=denoiser.x2 if warm else None, tv_u2=denoiser.u2 if warm else None)

        def run_fused(n):
            eng.run(n, graph_steps=graph_steps if n >= 2 * graph_steps else 0)

        if snaps is None:
            run_fused(n_iter)
        else:
            def snap(i):
                # Y_i of the step just run, recomputed from its input X_i (still in the ping-pong buffer)
                Xi = eng.input_state(i).contiguous()
                Yi = K.langevin_update(Xi, K.inpaint_grad(Xi, data_grad.y, data_grad.mask_u8, data_grad.sigma2),
                                       c1, c2, seed, chain0, i)
                snaps.save(i, eng.X, Yi, eng.lists())
            _run_with_snapshots(run_fused, n_iter, Kfreq, snap)
        eng.check_handoff()
        denoiser.x2 = eng.x2_state.contiguous().clone()
        denoiser.u2 = eng.u2_state.contiguous().clone()
        denoiser.restart = False
        return eng.lists()

    typed = isinstance(data_grad, (InpaintingFidelity, BlurFidelity))
    if typed and isinstance(denoiser, torch.nn.Module) and not isinstance(denoiser, TVDenoiser):
        sig_den = torch.tensor(sig_noised).to(dev).to(torch.float32)
        eng = DenoiserChains(X0, data_grad, denoiser, sig_den, alpha=alpha_f, c1=c1, c2=c2, seed=seed,
                             n_iter=n_iter, n_inter=n_inter, n_inter_mmse=n_inter_mmse, chain0=chain0)
        capturable = isinstance(denoiser, (DnCNN, DRUNet)) or getattr(denoiser, "capturable", False)

        def run_dnn(n):
            eng.run(n, graph_steps=graph_steps if (capturable and n >= 2 * graph_steps) else 0)

        if snaps is None:
            run_dnn(n_iter)
        else:
            def run_until_snapshot(n):
                run_dnn(n - 1)
                if n > 0:
                    eng.step_keep_state()       # the snapshot step: X_{i+1} materialised, Y_i kept

            def snap(i):
                snaps.save(i, eng.X_state, eng.Y_prev, _lists(eng.sched, eng.steps_done))
            done = 0
            for i in range(0, n_iter, Kfreq):
                run_until_snapshot(i + 1 - done)
                done = i + 1
                snap(i)
            run_dnn(n_iter - done)
        return _lists(eng.sched, eng.steps_done)

    # ---- generic path: opaque closures, HIP noise / update / relaxation / accumulators ----
    sched = K.Schedule(shape, n_iter, n_inter, n_inter_mmse, dev)
    X = X0
    Xn = torch.empty_like(X)
    Y = torch.empty_like(X)
    mean = torch.zeros_like(X)
    sq = torch.zeros_like(X)
    sig_den = torch.tensor(sig_noised).to(dev).to(torch.float32)
    tv_batch = isinstance(denoiser, TVDenoiser)
    with torch.no_grad():
        blur = isinstance(data_grad, BlurFidelity)
        for i in range(n_iter):
            if blur:    # deblurring: gradient stencil and Langevin update in one HIP kernel
                K.blur_langevin(X, data_grad.y.contiguous(), data_grad.taps_conv, data_grad.taps_corr, data_grad.l,
                                data_grad.sigma2, c1, c2, seed, chain0, i, out=Y, exact=data_grad.exact)
            else:
                g = data_grad(X)
                K.langevin_update(X, g.contiguous().float(), c1, c2, seed, chain0, i, out=Y)
            # a TV prox over B chains: deepinv's early stop per chain (each chain is one reference run)
            D = denoiser.forward(Y, sig_den, per_chain=True) if tv_batch else denoiser.forward(Y, sig_den)
            K.relax_accumulate(Y, D.contiguous(), Xn, alpha_f, mean, sq, sched, i)
            X, Xn = Xn, X
            if i % Kfreq == 0 and snaps is not None:
                snaps.save(i, X, Y, _lists(sched, i + 1))
    return _lists(sched, n_iter)


def pnpula(init, data_grad, prior_grad, delta, lambd, n_iter=5000, n_inter=1000, n_inter_mmse=1000, seed=None,
           device=None, c_min=-1, c_max=2, path=None, save_images_online=False, name=None, *, chain0: int = 0,
           graph_steps: int | None = None):
    """PnP-ULA (restoration_algorithms.py:38-160)."""
    if not init.is_cuda:
        raise ValueError("pnpula runs on the GPU: init must be a CUDA (HIP) tensor")
    delta_t = torch.as_tensor(delta).detach().to(torch.float32)
    brw = float(torch.sqrt((2 * delta_t.cpu()).double()).float().item())   # CUDA sqrtf: correctly rounded
    print("delta = {}".format(delta_t.float()))
    path = "" if path is None else path
    name = "" if name is None else name
    n_inter, n_inter_mmse, Kfreq = _check_schedule(n_iter, n_inter, n_inter_mmse, seed)
    dev = init.device
    X = init.clone().detach().contiguous().float()
    shape = X.shape
    d = float(delta_t.cpu().item())
    lam = float(torch.as_tensor(lambd).detach().cpu().to(torch.float32).item())
    if graph_steps is None:
        graph_steps = DEFAULT_GRAPH_STEPS
    snaps = None
    if save_images_online:
        snaps = _Snapshots(path, name, {"n_iter": n_iter, "c_min": c_min, "c_max": c_max, "lambda": lambd,
                                        "delta": delta})
    if isinstance(prior_grad, DenoiserPrior) and isinstance(data_grad, (InpaintingFidelity, BlurFidelity)):
        eng = UlaChains(X, data_grad, prior_grad, delta=d, lambd=lam, brw=brw, c_min=float(c_min),
                        c_max=float(c_max), seed=int(seed), n_iter=n_iter, n_inter=n_inter,
                        n_inter_mmse=n_inter_mmse, chain0=chain0)
        capturable = isinstance(prior_grad.denoiser, (DnCNN, DRUNet)) or getattr(prior_grad.denoiser, "capturable",
                                                                                False)

        def run_ula(n):
            eng.run(n, graph_steps=graph_steps if (capturable and n >= 2 * graph_steps) else 0)

        if snaps is None:
            run_ula(n_iter)
        else:
            _run_with_snapshots(run_ula, n_iter, Kfreq,
                                lambda i: snaps.save(i, eng.state, None, _lists(eng.sched, eng.steps_done)))
        return _lists(eng.sched, eng.steps_done)
    sched = K.Schedule(shape, n_iter, n_inter, n_inter_mmse, dev)
    Xn = torch.empty_like(X)
    mean = torch.zeros_like(X)
    sq = torch.zeros_like(X)
    with torch.no_grad():
        for i in range(n_iter):
            gp = prior_grad(X).contiguous().float()
            gd = data_grad(X).contiguous().float()
            K.pnpula_update(X, gp, gd, Xn, d, lam, brw, float(c_min), float(c_max), mean, sq, sched, i,
                            int(seed), chain0)
            X, Xn = Xn, X
            if i % Kfreq == 0 and snaps is not None:
                snaps.save(i, X, None, _lists(sched, i + 1))
    return _lists(sched, n_iter)
