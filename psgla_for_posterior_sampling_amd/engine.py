"""Batched, graph-replayable PSGLA engines over the fused HIP steps.

``FusedTvChains`` runs B independent PSGLA chains (inpainting fidelity + warm-started TV
prox) with one fused kernel launch per Langevin step (the band kernel adds a small finaliser):
restoration_algorithms.py:231-271 with the closures of sampling_images.py:295 and the
deepinv TVDenoiser of sampling_images.py:138.  All step-dependent quantities (noise
counter, block coefficients, sample / block slots, ping-pong parity) are derived on the
device from a step counter, so any number of steps can be captured once in a hipGraph
(``torch.cuda.CUDAGraph``) and replayed.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as N
from . import hip_ops as K


# PsglaTvStep.kernel_variant (include/psgla_hip.h)
KERNEL_VARIANTS = {"auto": 0, "band": 1, "stream": 2, "tile": 4}


class FusedTvChains:
    def __init__(self, init: torch.Tensor, y: torch.Tensor, mask_u8: torch.Tensor, *, c1: float, c2: float,
                 sigma2: float, alpha: float, ths: float, tv: K.TvConstants, seed: int, n_iter: int,
                 n_inter: int, n_inter_mmse: int, chain0: int = 0, exact: bool = False,
                 tv_x2: torch.Tensor | None = None, tv_u2: torch.Tensor | None = None,
                 store_samples: bool = True, store_blocks: bool = True, kernel_variant: str = "auto",
                 stream_wgs: int = 0, stream_windows: str = "auto", parallel_redo: bool = True):
        if init.dim() != 4:
            raise ValueError("init must be (B, C, H, W)")
        if tv.n_it > N.TV_MAX_FUSED_IT:
            raise ValueError(f"fused TV step supports n_it_max <= {N.TV_MAX_FUSED_IT}")
        dev = init.device
        B, C, H, Wd = init.shape
        self.shape = (B, C, H, Wd)
        self.W = Wd
        # rows padded to a multiple of 4 columns so that every width runs on the streaming kernel
        # (csrc/tv_stream.hip, tv_tile.hip: ldw); the padding columns are scratch and every result is a view
        # of the first W columns
        if kernel_variant not in KERNEL_VARIANTS:
            raise ValueError(f"kernel_variant must be one of {sorted(KERNEL_VARIANTS)}")
        self.ldw = Wd if (Wd % 4 == 0 or kernel_variant == "band") else (Wd + 3) // 4 * 4
        self.pshape = (B, C, H, self.ldw)
        self.device = dev
        self.alpha = float(alpha)
        self.alpha1 = self.alpha == 1.0
        f32 = dict(dtype=torch.float32, device=dev)
        self.x = [self._padded(init), torch.zeros(self.pshape, **f32)]
        self.u2 = [torch.zeros(self.pshape + (2,), **f32), torch.zeros(self.pshape + (2,), **f32)]
        self.mean = [torch.zeros(self.pshape, **f32), torch.zeros(self.pshape, **f32)]
        self.sq = [torch.zeros(self.pshape, **f32), torch.zeros(self.pshape, **f32)]
        self.x2 = None
        warm = tv_x2 is not None and tuple(tv_x2.shape) == self.shape
        if not self.alpha1 or warm:
            self.x2 = [torch.zeros(self.pshape, **f32), torch.zeros(self.pshape, **f32)]
        if warm:
            self.x2[0][..., :Wd].copy_(tv_x2)
            self.u2[0][..., :Wd, :].copy_(tv_u2)
        self.y = self._padded(y)
        self.mask = self._padded(mask_u8)
        self.sched = K.Schedule(self.pshape, n_iter, n_inter, n_inter_mmse, dev, store_samples, store_blocks)
        # rel-err partial sums spread over 8 copies (one per XCD) for the tile kernel: one image's 246 tiles
        # no longer queue on the same 16 atomics (castle B = 1: DESIGN.md 3.1b)
        self.work = K.TvWorkspace(B, tv.n_it, dev, copies=8)
        self.work.fresh.fill_(0 if warm else 1)
        self.steps_done = 0
        self.n_iter = int(n_iter)
        self.warm_first = warm and self.alpha1

        d = N.PsglaTvStep()
        d.B, d.C, d.H, d.W = B, C, H, Wd
        d.ldw = self.ldw
        for i in range(2):
            d.x[i] = self.x[i].data_ptr()
            d.u2[i] = self.u2[i].data_ptr()
            d.mean[i] = self.mean[i].data_ptr()
            d.sq[i] = self.sq[i].data_ptr()
            d.x2[i] = self.x2[i].data_ptr() if (self.x2 is not None and not self.alpha1) else None
        d.y = K._ptr(self.y, name="y")
        d.y_chain_stride = 0 if self.y.shape[0] == 1 else C * H * self.ldw
        d.mask = K._ptr(self.mask, torch.uint8, "mask")
        d.mask_chain_stride = 0 if (self.mask.dim() == 2 or self.mask.shape[0] == 1) else H * self.ldw
        d.c1, d.c2, d.sigma2, d.alpha = c1, c2, sigma2, self.alpha
        d.tau, d.one_plus_tau, d.sigma_tv, d.rho = tv.tau, tv.one_plus_tau, tv.sigma_tv, tv.rho
        d.ths = float(np.float32(ths))
        d.tol = tv.tol
        d.n_tv = tv.n_it
        d.exact = int(bool(exact))
        d.seed = int(seed) & (2 ** 64 - 1)
        d.chain0 = int(chain0)
        d.advance_step = 1
        d.fresh = self.work.fresh.data_ptr()
        d.norms = self.work.norms_all.data_ptr()
        d.norms_copies = self.work.copies
        d.arrive = self.work.arrive.data_ptr()
        d.kernel_variant = KERNEL_VARIANTS[kernel_variant]
        d.stream_wgs = int(stream_wgs)
        if stream_windows not in ("auto", "whole", "half"):
            raise ValueError("stream_windows must be 'auto', 'whole' or 'half'")
        d.stream_windows = {"auto": 0, "whole": 1, "half": 2}[stream_windows]
        # deepinv's early stop, when it fires, is redone in parallel by the next launch (include/psgla_hip.h); the
        # last step's pending redo is settled (launch_mask 4) before results are read: settle()
        d.redo = self.work.redo.data_ptr() if parallel_redo else None
        self.desc = d
        self._unsettled = False
        self.sched_struct = self.sched.struct(True, 0)
        if self.warm_first:
            # first step of a warm-started run: the TV primal x2 (previous run's state) is not X
            d0 = N.PsglaTvStep.from_buffer_copy(d)
            d0.x2[0] = self.x2[0].data_ptr()
            d0.x2[1] = self.x2[1].data_ptr()
            self.desc_first = d0
        self.graph = None
        self.graph_steps = 0

    def _padded(self, t: torch.Tensor) -> torch.Tensor:
        """Contiguous copy of t (..., W) with rows padded by zeros to the row pitch ldw."""
        t = t.contiguous()
        if self.ldw == self.W:
            return t.clone()
        out = torch.zeros(t.shape[:-1] + (self.ldw,), dtype=t.dtype, device=t.device)
        out[..., :self.W].copy_(t)
        return out

    def _view(self, t: torch.Tensor, u2: bool = False) -> torch.Tensor:
        if t is None or self.ldw == self.W:
            return t
        return t[..., :self.W, :] if u2 else t[..., :self.W]

    # -- stepping -----------------------------------------------------------------
    def _launch(self, desc):
        N.check(N.lib().psgla_tv_step(ctypes.byref(desc), ctypes.byref(self.sched_struct), K._stream()),
                "psgla_tv_step")

    def step(self, n: int = 1):
        """Launch n steps eagerly (async on the current stream)."""
        for _ in range(n):
            if self.steps_done >= self.n_iter:
                raise RuntimeError("all n_iter steps already done")
            if self.steps_done == 0 and self.warm_first:
                self._launch(self.desc_first)
                self.steps_done += 1
                # a warm-started first step reads the previous run's TV primal (desc_first's x2): its redo, if any,
                # must run with that descriptor, not with the next step's
                self._unsettled = True
                self.settle(self.desc_first)
                continue
            self._launch(self.desc)
            self.steps_done += 1
            self._unsettled = True

    def settle(self, desc=None):
        """Apply a pending early-stop redo of the last step (launch_mask 4: the stopped chains' part of that
        step, recomputed in parallel; nothing when no chain stopped).  Every result accessor calls it."""
        desc = self.desc if desc is None else desc
        if self._unsettled and desc.redo:
            d = N.PsglaTvStep.from_buffer_copy(desc)
            d.launch_mask = 4
            self._launch(d)
        self._unsettled = False

    def capture(self, steps_per_graph: int):
        """Capture `steps_per_graph` identical steps into one hipGraph (after step 0): one launch per
        step."""
        if self.steps_done == 0 and self.warm_first:
            self.step(1)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(steps_per_graph):
                self._launch(self.desc)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = g
        self.graph_steps = steps_per_graph

    def replay(self, times: int = 1):
        for _ in range(times):
            if self.steps_done + self.graph_steps > self.n_iter:
                raise RuntimeError("replay would exceed n_iter")
            self.graph.replay()
            self.steps_done += self.graph_steps
            self._unsettled = True

    def rewind(self, step: int, discard_pending: bool = False):
        """Set the step index (device counter, stream-ordered, and host count) back to `step`, which
        must have the parity of the current step (the ping-pong state stays where it is).  For
        benchmarking only: untimed warm-up replays can then run for any length of time and the timed
        steps still write the sample / block slots of the schedule (the chain state simply continues).
        discard_pending: drop a pending early-stop redo instead of settling it (warm-up replays whose state
        restore() undoes: no redo-only launch per replay in a kernel trace)."""
        step = int(step)
        if step < 0 or (step - self.steps_done) % 2:
            raise ValueError("rewind target must be >= 0 and of the current step's parity")
        if discard_pending:
            self.work.redo.zero_()
            self._unsettled = False
        else:
            self.settle()                 # a pending redo belongs to the step before the rewind
        self.sched.d_step.fill_(step)
        self.steps_done = step

    def snapshot(self) -> dict:
        """Device copies of everything a step reads or advances (chain / TV state, live accumulators, the
        step counter, the TV restart flag) -- for benchmarking: replays after a snapshot can be undone by
        restore() (samples / block means already written stay written)."""
        self.settle()
        torch.cuda.current_stream().synchronize()
        bufs = {"x": self.x, "u2": self.u2, "mean": self.mean, "sq": self.sq}
        if self.x2 is not None:
            bufs["x2"] = self.x2
        snap = {k: [t.clone() for t in v] for k, v in bufs.items()}
        snap["d_step"] = self.sched.d_step.clone()
        snap["fresh"] = self.work.fresh.clone()
        snap["steps_done"] = self.steps_done
        return snap

    def restore(self, snap: dict):
        torch.cuda.current_stream().synchronize()
        for k in ("x", "u2", "mean", "sq", "x2"):
            if k in snap:
                for dst, src in zip(getattr(self, k), snap[k]):
                    dst.copy_(src)
        self.sched.d_step.copy_(snap["d_step"])
        self.work.fresh.copy_(snap["fresh"])
        self.work.redo.zero_()            # snapshots are settled: nothing pending
        self.steps_done = snap["steps_done"]
        self._unsettled = False

    @property
    def main_kernel(self) -> str:
        """Name of the kernel psgla_tv_step dispatches for this shape (the library's own choice,
        psgla_tv_step_kernel: the small-batch tile kernel when its tiles fit on the CUs at once, else
        the row stream (W % 4 == 0 rows -- always, the engine pads rows --, 1 <= n_tv <= 10, H >= 2); the band
        kernel otherwise or when forced)."""
        k = N.lib().psgla_tv_step_kernel(ctypes.byref(self.desc))
        if k < 0:
            raise RuntimeError(N.lib().psgla_last_error().decode())
        return {0: "tv_main_kernel", 1: "tv_stream_kernel", 3: "tv_tile_kernel"}[k]

    def launch_main_only(self, n: int = 1):
        """Launch only the fused tile kernel n times for the CURRENT step (idempotent: it reads
        the step's inputs and rewrites the same outputs; the step counter does not move).
        Used to time the dominant kernel alone.  A pending early-stop redo of the last step is settled first:
        this launch rewrites the ping-pong buffer that redo reads its inputs from."""
        self.settle()
        d = N.PsglaTvStep.from_buffer_copy(self.desc)
        d.launch_mask = 1
        for _ in range(n):
            self._launch(d)

    def run(self, n: int | None = None, graph_steps: int = 0):
        n = self.n_iter - self.steps_done if n is None else n
        if graph_steps > 0 and n >= graph_steps:
            if self.steps_done == 0 and self.warm_first:
                self.step(1)
                n -= 1
            if self.graph is None or self.graph_steps != graph_steps:
                self.capture(graph_steps)
            reps = n // graph_steps
            self.replay(reps)
            n -= reps * graph_steps
        self.step(n)

    def check_handoff(self):
        """Raise if an early-stop recompute ever gave up waiting for the other workgroups (arrive[3],
        include/psgla_hip.h: the tile kernel's serial recompute waiting for their stores, or the parallel redo's
        grid barrier; guards that should never expire -- if one did, the recomputed chains may have raced the
        other workgroups' stores).  One host sync."""
        self.settle()
        if int(self.work.arrive[3].item()) != 0:
            raise RuntimeError("early-stop recompute hand-off guard expired (tv_stream_kernel / tv_tile_kernel); "
                               "results of the recomputed chains are not trustworthy")

    # -- results --------------------------------------------------------------------
    @property
    def X(self) -> torch.Tensor:
        self.settle()
        return self._view(self.x[self.steps_done & 1])

    def input_state(self, step: int) -> torch.Tensor:
        """X_step, the input of step `step` -- intact in its ping-pong buffer until step + 1 has run."""
        if not (self.steps_done - 1 <= step <= self.steps_done):
            raise ValueError("only the last step's input is still held")
        if step == self.steps_done:
            self.settle()           # the last step's output: a pending early-stop redo rewrites it
        return self._view(self.x[step & 1])

    @property
    def u2_state(self) -> torch.Tensor:
        self.settle()
        return self._view(self.u2[self.steps_done & 1], u2=True)

    @property
    def x2_state(self) -> torch.Tensor:
        if self.alpha1:
            return self.X
        self.settle()
        return self._view(self.x2[self.steps_done & 1])

    def samples(self):
        self.settle()
        if self.sched.samples is None:
            return None
        k = self.sched.n_samples_done(self.steps_done)
        return self._view(self.sched.samples[:k])

    def blocks(self):
        self.settle()
        k = self.sched.n_blocks_done(self.steps_done)
        if self.sched.blocks is None:
            return None, None
        return self._view(self.sched.blocks[:k]), self._view(self.sched.blocks2[:k])

    def lists(self):
        """The reference's return value: lists of squeezed (C, H, W) tensors (views of the stores).  Checks the
        early-stop hand-off guard first (check_handoff: settles, one host sync -- the results are being read;
        ADVICE r5: not only in psgla())."""
        self.check_handoff()
        ns = self.sched.n_samples_done(self.steps_done)
        nb = self.sched.n_blocks_done(self.steps_done)
        sm, (b1, b2) = self.samples(), self.blocks()
        Xlist = [torch.squeeze(sm[k]) for k in range(ns)] if sm is not None else []
        M = [torch.squeeze(b1[k]) for k in range(nb)] if b1 is not None else []
        M2 = [torch.squeeze(b2[k]) for k in range(nb)] if b2 is not None else []
        return Xlist, M, M2


def _capture(body, k: int, device):
    """Record `k` calls of `body` into one hipGraph (torch.cuda.CUDAGraph) on a side stream."""
    s = torch.cuda.Stream(device=device)
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(k):
            body()
    torch.cuda.current_stream().wait_stream(s)
    return g


class _GraphRunner:
    """Eager / graph-replayed stepping shared by the DNN engines.  Buffer roles alternate by step
    parity, so a graph holds an even number of steps and leaves them where it found them."""

    steps_done: int
    n_iter: int

    def _body(self):  # pragma: no cover - abstract
        raise NotImplementedError

    def step(self, n: int = 1):
        with torch.no_grad():
            for _ in range(n):
                if self.steps_done >= self.n_iter:
                    raise RuntimeError("all n_iter steps already done")
                self._body()
                self.steps_done += 1

    def capture(self, steps_per_graph: int):
        k = steps_per_graph + (steps_per_graph & 1)
        self.graph_cur = self.cur          # the buffer parity the recorded pointers assume
        with torch.no_grad():
            self.graph = _capture(self._body, k, self.device)
        self.graph_steps = k

    def replay(self, times: int = 1):
        for _ in range(times):
            if self.steps_done + self.graph_steps > self.n_iter:
                raise RuntimeError("replay would exceed n_iter")
            self.graph.replay()
            self.steps_done += self.graph_steps

    def run(self, n: int | None = None, graph_steps: int = 0):
        n = self.n_iter - self.steps_done if n is None else n
        if self.steps_done < 2:
            # two eager steps first: the denoiser's kernels (MIOpen) pick their algorithms outside capture
            warm = min(n, 2 - self.steps_done)
            self.step(warm)
            n -= warm
        if graph_steps > 0 and n >= graph_steps:
            if self.graph is None or self.graph_steps != graph_steps + (graph_steps & 1):
                self.capture(graph_steps)
            if self.cur != self.graph_cur:
                # an odd number of eager steps since the capture: one more, so the replayed pointers
                # (recorded at parity graph_cur) see the buffers they were recorded with
                self.step(1)
                n -= 1
            reps = n // self.graph_steps
            self.replay(reps)
            n -= reps * self.graph_steps
        self.step(n)


class DenoiserChains(_GraphRunner):
    """B PSGLA chains with a PyTorch denoiser (DnCNN / DRUNet forward on PyTorch-ROCm) and a typed data
    term: restoration_algorithms.py:231-271 with sampling_images.py:295 (inpainting) or :329-338
    (deblurring).  Per step: ``D = denoiser.forward(Y, sigma)`` and then
      inpainting: ONE HIP pass -- relaxation, accumulators / samples of step i and the next step's
                  Langevin update Y' = (X + c1 g(X)) + c2 Z_{i+1}  (psgla_relax_langevin_inpaint);
      deblurring: relaxation + accumulators, then the stencil kernel with the Langevin update fused.
    The step index lives on the device, so steps [denoiser + HIP passes] are captured in one hipGraph
    and replayed.  Identical results to the reference's loop order (the denoiser sees Y_i; X_{i+1}
    is accumulated with step index i)."""

    def __init__(self, init: torch.Tensor, data_grad, denoiser, sig_den, *, alpha: float, c1: float, c2: float,
                 seed: int, n_iter: int, n_inter: int, n_inter_mmse: int, chain0: int = 0):
        from .fidelity import BlurFidelity, InpaintingFidelity
        if init.dim() != 4:
            raise ValueError("init must be (B, C, H, W)")
        self.inpaint = isinstance(data_grad, InpaintingFidelity)
        if not (self.inpaint or isinstance(data_grad, BlurFidelity)):
            raise TypeError("DenoiserChains needs an InpaintingFidelity or a BlurFidelity data term")
        B, C, H, W = init.shape
        self.device = init.device
        self.shape = (B, C, H, W)
        self.fid = data_grad
        self.denoiser = denoiser
        self.sig = sig_den
        self.alpha = float(alpha)
        self.c1, self.c2 = float(c1), float(c2)
        self.seed, self.chain0 = int(seed), int(chain0)
        self.n_iter = int(n_iter)
        X0 = init.contiguous().float()
        self.Y = [torch.empty_like(X0), torch.empty_like(X0)]
        self.X = None if self.inpaint else torch.empty_like(X0)
        self._keep = False          # step_keep_state(): materialise X_{i+1} (inpainting writes it only then)
        self._Xsnap = None
        self.mean = torch.zeros_like(X0)
        self.sq = torch.zeros_like(X0)
        self.sched = K.Schedule(self.shape, n_iter, n_inter, n_inter_mmse, self.device)
        self.cur = 0
        self.steps_done = 0
        self.graph = None
        self.graph_steps = 0
        # prologue: Y_0 = (X_0 + c1 g(X_0)) + c2 Z_0
        if self.inpaint:
            g = K.inpaint_grad(X0, data_grad.y, data_grad.mask_u8, data_grad.sigma2)
            K.langevin_update(X0, g, self.c1, self.c2, self.seed, self.chain0, 0, out=self.Y[0])
        else:
            f = data_grad
            K.blur_langevin(X0, f.y.contiguous(), f.taps_conv, f.taps_corr, f.l, f.sigma2, self.c1, self.c2,
                            self.seed, self.chain0, 0, out=self.Y[0], exact=f.exact)

    def _body(self):
        Yc, Yn = self.Y[self.cur], self.Y[1 - self.cur]
        D = self.denoiser.forward(Yc, self.sig).contiguous().float()
        f = self.fid
        if self.inpaint:
            xo = None
            if self._keep:
                if self._Xsnap is None:
                    self._Xsnap = torch.empty_like(Yc)
                xo = self._Xsnap
            K.relax_langevin_inpaint(Yc, D, self.alpha, f.y, f.mask_u8, f.sigma2, self.c1, self.c2, self.seed,
                                     self.chain0, self.mean, self.sq, self.sched, 0, Yn, X_out=xo,
                                     use_device_step=True)
        else:
            K.relax_accumulate(Yc, D, self.X, self.alpha, self.mean, self.sq, self.sched, 0, use_device_step=True)
            K.blur_langevin(self.X, f.y.contiguous(), f.taps_conv, f.taps_corr, f.l, f.sigma2, self.c1, self.c2,
                            self.seed, self.chain0, 1, out=Yn, exact=f.exact, d_step=self.sched.d_step)
        K.advance_step(self.sched.d_step)
        self.cur ^= 1

    def step_keep_state(self):
        """One eager step i that also keeps what save_images_online shows (restoration_algorithms.py:246-253):
        X_{i+1} (``X_state``) and the step's Langevin proposal Y_i (``Y_prev``)."""
        self._keep = True
        try:
            self.step(1)
        finally:
            self._keep = False

    @property
    def X_state(self) -> torch.Tensor:
        """X after the last step run by step_keep_state() (inpainting) / the last step (deblurring)."""
        return self._Xsnap if self.inpaint else self.X

    @property
    def Y_prev(self) -> torch.Tensor:
        """Y_i of the last step run (the buffer the next step overwrites)."""
        return self.Y[1 - self.cur]


class UlaChains(_GraphRunner):
    """B PnP-ULA chains (restoration_algorithms.py:102-144) with a capturable prior gradient (e.g.
    :class:`~psgla_for_posterior_sampling_amd.denoisers.DenoiserPrior` over DRUNet / DnCNN) and a
    typed data term: per step the prior and data gradients, then one HIP pass (projection, update,
    noise, accumulators); the step index lives on the device, so steps are hipGraph-replayed."""

    def __init__(self, init: torch.Tensor, data_grad, prior_grad, *, delta: float, lambd: float, brw: float,
                 c_min: float, c_max: float, seed: int, n_iter: int, n_inter: int, n_inter_mmse: int,
                 chain0: int = 0):
        self.device = init.device
        X0 = init.contiguous().float().clone()
        self.shape = tuple(X0.shape)
        self.X = [X0, torch.empty_like(X0)]
        self.mean = torch.zeros_like(X0)
        self.sq = torch.zeros_like(X0)
        self.data_grad, self.prior_grad = data_grad, prior_grad
        self.delta, self.lambd, self.brw = float(delta), float(lambd), float(brw)
        # V-ULA: a DenoiserPrior's arithmetic (alpha (D - x) / s2), the data term and the update in one
        # HIP pass after the denoiser forward (the scalars read once here, outside any capture)
        from .denoisers import DenoiserPrior
        from .fidelity import BlurFidelity, InpaintingFidelity
        self.fused = isinstance(prior_grad, DenoiserPrior) and isinstance(data_grad, (InpaintingFidelity, BlurFidelity))
        if self.fused:
            self.alpha_f = float(torch.as_tensor(prior_grad.alpha).float().item())
            self.s2_f = float(torch.as_tensor(prior_grad.s2).float().item())
            self.inpaint = isinstance(data_grad, InpaintingFidelity)
        self.c_min, self.c_max = float(c_min), float(c_max)
        self.seed, self.chain0 = int(seed), int(chain0)
        self.n_iter = int(n_iter)
        self.sched = K.Schedule(self.shape, n_iter, n_inter, n_inter_mmse, self.device)
        self.cur = 0
        self.steps_done = 0
        self.graph = None
        self.graph_steps = 0

    def _body(self):
        X, Xn = self.X[self.cur], self.X[1 - self.cur]
        if self.fused:
            p, f = self.prior_grad, self.data_grad
            D = p.denoiser.forward(X, p.s1).contiguous().float()
            if self.inpaint:
                K.pnpula_prior_update(X, D, self.alpha_f, self.s2_f, Xn, self.delta, self.lambd, self.brw, self.c_min,
                                      self.c_max, self.mean, self.sq, self.sched, 0, self.seed, self.chain0, y=f.y,
                                      mask_u8=f.mask_u8, sigma2=f.sigma2, use_device_step=True)
            else:
                gd = f(X).contiguous().float()
                K.pnpula_prior_update(X, D, self.alpha_f, self.s2_f, Xn, self.delta, self.lambd, self.brw, self.c_min,
                                      self.c_max, self.mean, self.sq, self.sched, 0, self.seed, self.chain0, gd=gd,
                                      use_device_step=True)
        else:
            gp = self.prior_grad(X).contiguous().float()
            gd = self.data_grad(X).contiguous().float()
            K.pnpula_update(X, gp, gd, Xn, self.delta, self.lambd, self.brw, self.c_min, self.c_max, self.mean,
                            self.sq, self.sched, 0, self.seed, self.chain0, use_device_step=True)
        K.advance_step(self.sched.d_step)
        self.cur ^= 1

    @property
    def state(self) -> torch.Tensor:
        return self.X[self.cur]
