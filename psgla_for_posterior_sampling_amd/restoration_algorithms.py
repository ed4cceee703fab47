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
The Gaussian noise is the in-kernel "psgla noise v1" stream of (seed, chain) instead of
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


def _save_online(path, name, i, X, Y, sched, steps_done, extra):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    xn = np.transpose(X.detach().cpu().numpy()[0], (1, 2, 0))
    plt.imsave(path + "/x_" + str(i) + ".png", np.clip(xn, 0, 1), cmap=None)
    if Y is not None:
        yn = np.transpose(Y.detach().cpu().numpy()[0], (1, 2, 0))
        plt.imsave(path + "/y_" + str(i) + ".png", np.clip(yn, 0, 1), cmap=None)
    Xl, M, M2 = _lists(sched, steps_done)
    d = {"Samples": Xl, "Mmse": M, "Mmse2": M2}
    d.update(extra)
    torch.save(d, path + "/" + name + "_sampling.pth")


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

    fused = (isinstance(data_grad, InpaintingFidelity) and isinstance(denoiser, TVDenoiser)
             and denoiser.n_it_max <= K.N.TV_MAX_FUSED_IT and not save_images_online)
    if fused:
        if exact is None:
            exact = denoiser.exact
        warm = not denoiser.needs_restart(shape)
        eng = FusedTvChains(X0, data_grad.y, data_grad.mask_u8, c1=c1, c2=c2, sigma2=data_grad.sigma2,
                            alpha=alpha_f, ths=float(np.float32(sig_noised)), tv=denoiser.constants(), seed=seed,
                            n_iter=n_iter, n_inter=n_inter, n_inter_mmse=n_inter_mmse, chain0=chain0,
                            exact=exact, tv_x2=denoiser.x2 if warm else None, tv_u2=denoiser.u2 if warm else None)
        eng.run(n_iter, graph_steps=graph_steps if n_iter >= 2 * graph_steps else 0)
        denoiser.x2 = eng.x2_state.contiguous().clone()
        denoiser.u2 = eng.u2_state.contiguous().clone()
        denoiser.restart = False
        return eng.lists()

    typed = isinstance(data_grad, (InpaintingFidelity, BlurFidelity))
    if (typed and isinstance(denoiser, torch.nn.Module) and not isinstance(denoiser, TVDenoiser)
            and not save_images_online and not (isinstance(data_grad, InpaintingFidelity)
                                                and (shape[2] * shape[3]) % 4)):
        sig_den = torch.tensor(sig_noised).to(dev).to(torch.float32)
        eng = DenoiserChains(X0, data_grad, denoiser, sig_den, alpha=alpha_f, c1=c1, c2=c2, seed=seed,
                             n_iter=n_iter, n_inter=n_inter, n_inter_mmse=n_inter_mmse, chain0=chain0)
        capturable = isinstance(denoiser, (DnCNN, DRUNet)) or getattr(denoiser, "capturable", False)
        eng.run(n_iter, graph_steps=graph_steps if (capturable and n_iter >= 2 * graph_steps) else 0)
        return _lists(eng.sched, eng.steps_done)

    # ---- generic path: opaque closures, HIP noise / update / relaxation / accumulators ----
    sched = K.Schedule(shape, n_iter, n_inter, n_inter_mmse, dev)
    X = X0
    Xn = torch.empty_like(X)
    Y = torch.empty_like(X)
    mean = torch.zeros_like(X)
    sq = torch.zeros_like(X)
    sig_den = torch.tensor(sig_noised).to(dev).to(torch.float32)
    with torch.no_grad():
        blur = isinstance(data_grad, BlurFidelity)
        for i in range(n_iter):
            if blur:    # deblurring: gradient stencil and Langevin update in one HIP kernel
                K.blur_langevin(X, data_grad.y.contiguous(), data_grad.taps_conv, data_grad.taps_corr, data_grad.l,
                                data_grad.sigma2, c1, c2, seed, chain0, i, out=Y, exact=data_grad.exact)
            else:
                g = data_grad(X)
                K.langevin_update(X, g.contiguous().float(), c1, c2, seed, chain0, i, out=Y)
            D = denoiser.forward(Y, sig_den)
            K.relax_accumulate(Y, D.contiguous(), Xn, alpha_f, mean, sq, sched, i)
            X, Xn = Xn, X
            if i % Kfreq == 0 and save_images_online:
                _save_online(path, name, i, X, Y, sched, i + 1,
                             {"n_iter": n_iter, "lambda": lambd, "delta": delta_t.to(dev)})
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
    if (isinstance(prior_grad, DenoiserPrior) and isinstance(data_grad, (InpaintingFidelity, BlurFidelity))
            and not save_images_online):
        eng = UlaChains(X, data_grad, prior_grad, delta=d, lambd=lam, brw=brw, c_min=float(c_min),
                        c_max=float(c_max), seed=int(seed), n_iter=n_iter, n_inter=n_inter,
                        n_inter_mmse=n_inter_mmse, chain0=chain0)
        capturable = isinstance(prior_grad.denoiser, (DnCNN, DRUNet)) or getattr(prior_grad.denoiser, "capturable",
                                                                                False)
        eng.run(n_iter, graph_steps=graph_steps if (capturable and n_iter >= 2 * graph_steps) else 0)
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
            if i % Kfreq == 0 and save_images_online:
                _save_online(path, name, i, X, None, sched, i + 1,
                             {"n_iter": n_iter, "c_min": c_min, "c_max": c_max, "lambda": lambd, "delta": delta})
    return _lists(sched, n_iter)
