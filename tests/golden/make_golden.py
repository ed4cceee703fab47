"""Generate the golden parity fixtures from the REFERENCE itself (run in the build
container only -- /root/reference does not exist on the GPU box).

    python tests/golden/make_golden.py

What is executed from the reference (read-only, never copied into the repo):

* ``restoration_algorithms.psgla`` / ``pnpula`` (restoration_algorithms.py:38, :163),
  imported as a module with the two unused module-level imports stubbed
  (``cv2`` :8 and ``deepinv.optim.data_fidelity.L2`` :9; neither is installed
  and neither is used by psgla/pnpula).  ``torch.randn`` inside that module is
  redirected to the psgla noise stream (oracle/noise.c; every fixture has W % 4 == 0,
  where the round-1 "v1" and the current "v2" numbering are one stream), so the reference
  consumes exactly the noise the HIP kernels generate.
* the data-fidelity set-up of sampling_images.py:283-341 and the parameter
  derivation of sampling_images.py:100-123 / :147-198, executed from the
  reference's own source text (that script is not importable: module-level
  argparse, deepinv, skimage, CUDA device).  The only textual patch is the
  device string ``"cuda:"+str(pars.gpu_number)`` -> ``"cpu"``.
* the TV denoiser is the deepinv 0.2.1 restatement in oracle/psgla_oracle.py
  (deepinv is not vendored/installable offline: TV arithmetic stays "parity
  unpinned" beyond this restatement).

Outputs: tests/golden/*.npz (inputs + reference outputs) and params.json.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import tempfile
import textwrap
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
from oracle import psgla_oracle as orc  # noqa: E402


# ---------------------------------------------------------------------------------------
def load_reference_algorithms():
    sys.modules.setdefault("cv2", types.ModuleType("cv2"))
    dv = types.ModuleType("deepinv")
    dvo = types.ModuleType("deepinv.optim")
    dvf = types.ModuleType("deepinv.optim.data_fidelity")
    dvf.L2 = object
    dv.optim = dvo
    dvo.data_fidelity = dvf
    for name, mod in (("deepinv", dv), ("deepinv.optim", dvo), ("deepinv.optim.data_fidelity", dvf)):
        sys.modules.setdefault(name, mod)
    spec = importlib.util.spec_from_file_location("ref_restoration_algorithms",
                                                  os.path.join(REF, "restoration_algorithms.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class NoiseInjectingTorch(types.ModuleType):
    """Proxy for the reference module's global ``torch``: ``randn`` returns the
    psgla-noise-v1 stream of (seed, chain) step by step; everything else is torch."""

    def __init__(self, seed: int, chain: int = 0):
        super().__init__("torch_proxy")
        self._seed = seed
        self._chain = chain
        self._step = 0

    def __getattr__(self, name):
        return getattr(torch, name)

    def randn(self, shape, generator=None, dtype=None, device=None):
        z = orc.normal(tuple(shape), self._seed, self._chain, self._step)
        self._step += 1
        return z


def reference_source(path: str, first: int, last: int) -> str:
    with open(os.path.join(REF, path)) as f:
        lines = f.readlines()[first - 1:last]
    return textwrap.dedent("".join(lines))


def reference_fidelity(Pb: str, im_t: torch.Tensor, **kw):
    """Execute sampling_images.py:283-341 on CPU for a given problem."""
    pars = types.SimpleNamespace(Pb=Pb, prop=kw.get("prop", 0.5), seed_ip=kw.get("seed_ip", 0),
                                 blur_type=kw.get("blur_type", "uniform"), si=kw.get("si", 1.0),
                                 grayscale=False)
    sigma = kw.get("sigma", 1.0)
    sigma1 = sigma / 255.0
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    tmp = tempfile.mkdtemp()
    ns = dict(torch=torch, np=np, plt=plt, pars=pars, im_t=im_t, device="cpu", sigma1=sigma1,
              sigma2t=torch.tensor(sigma1 ** 2, dtype=torch.float32), l=kw.get("l", 4),
              tensor=torch.FloatTensor, path_result_im=tmp)
    exec(compile(reference_source("sampling_images.py", 283, 341), "sampling_images.py:283", "exec"), ns)
    return ns


def reference_params(argv: list[str], **pars_kw):
    """Execute the constant derivation sampling_images.py:100-123 and :147-198."""
    defaults = dict(N=10000, alpha=1.0, s=5.0, sigma=1.0, l=4, delta=3e-5, lambd=1.0, seed_alg=0,
                    gpu_number=0, alg="psgla", den="DnCNN", Pb="inpainting", zeta=0.8, t_start=200)
    defaults.update(pars_kw)
    pars = types.SimpleNamespace(**defaults)
    src = reference_source("sampling_images.py", 100, 123) + reference_source("sampling_images.py", 147, 198)
    src = src.replace('"cuda:"+str(pars.gpu_number)', '"cpu"')

    class _Den:
        def forward(self, x, s):
            return x
    ns = dict(torch=torch, np=np, pars=pars, denoiser=_Den(), sys=types.SimpleNamespace(argv=argv))
    exec(compile(src, "sampling_images.py:100", "exec"), ns)
    out = {k: ns[k] for k in ("N", "n_inter", "s", "lambd", "delta_float") if k in ns}
    out["n_inter_mmse"] = int(ns["n_inter_mmse"])
    out["alpha"] = float(ns["alpha"])
    out["sigma2t"] = float(ns["sigma2t"])
    if "lambdt" in ns:
        out["lambdt"] = float(ns["lambdt"])
    if "deltat" in ns:
        out["deltat"] = float(ns["deltat"])
    if "s1" in ns:
        out["s1"] = float(ns["s1"])
    return {k: (float(v) if isinstance(v, (float, np.floating)) else v) for k, v in out.items()}


# ---------------------------------------------------------------------------------------
def ground_truth(C, H, W, seed=1234):
    g = torch.Generator().manual_seed(seed)
    return torch.rand((1, C, H, W), generator=g)


def stack(lst):
    return np.stack([t.numpy() for t in lst]).astype(np.float32) if lst else np.zeros((0,), np.float32)


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


def run_psgla(ra, init, data_grad, denoiser, alpha, lambd, s, delta, n_iter, n_inter, n_inter_mmse,
              seed):
    ra.torch = NoiseInjectingTorch(seed)
    try:
        return ra.psgla(init=init, data_grad=data_grad, denoiser=denoiser,
                        alpha=torch.tensor(alpha, dtype=torch.float32),
                        lambd=torch.tensor(lambd, dtype=torch.float32), sig_float=s, delta=delta,
                        seed=seed, device="cpu", n_iter=n_iter, n_inter=n_inter,
                        n_inter_mmse=n_inter_mmse)
    finally:
        ra.torch = torch


def run_pnpula(ra, init, data_grad, prior_grad, delta_t, lambd_t, n_iter, n_inter, n_inter_mmse,
               seed):
    ra.torch = NoiseInjectingTorch(seed)
    try:
        return ra.pnpula(init=init, data_grad=data_grad, prior_grad=prior_grad, delta=delta_t,
                         lambd=lambd_t, seed=seed, device="cpu", n_iter=n_iter, n_inter=n_inter,
                         n_inter_mmse=n_inter_mmse)
    finally:
        ra.torch = torch


def main():
    torch.set_num_threads(4)
    ra = load_reference_algorithms()
    params = {}

    # ---- parameter derivations (sampling_images.py:100-123, :147-198) -------------
    params["psgla_TV_defaults"] = reference_params(["sampling_images.py", "--alg", "psgla", "--den", "TV"],
                                                   alg="psgla", den="TV")
    params["psgla_TV_N10000"] = reference_params(
        ["sampling_images.py", "--alg", "psgla", "--den", "TV", "--N", "10000"], alg="psgla", den="TV")
    params["psgla_DnCNN_defaults"] = reference_params(["sampling_images.py"], alg="psgla", den="DnCNN")
    params["pnp_ula_DRUNet_N1e6"] = reference_params(
        ["sampling_images.py", "--alg", "pnp_ula", "--den", "DRUNet", "--N", "1000000"],
        alg="pnp_ula", den="DRUNet", N=1000000)
    params["pnp_ula_DnCNN_defaults"] = reference_params(["sampling_images.py", "--alg", "pnp_ula"],
                                                       alg="pnp_ula", den="DnCNN")

    # ---- (1) psgla + inpainting + clamp denoiser, 1x3x32x32 ----------------------
    x = ground_truth(3, 32, 32)
    ns = reference_fidelity("inpainting", x)
    p = params["psgla_DnCNN_defaults"]
    seed = 0
    Xl, Ml, M2l = run_psgla(ra, ns["init_torch"], ns["data_grad"], orc.ClampDenoiser(), 1.0, p["lambd"],
                            p["s"], p["delta_float"], 120, 10, 10, seed)
    save("psgla_inpaint_clamp", x=x.numpy(), y=ns["y_t"].numpy(), init=ns["init_torch"].numpy(),
         mask2d=ns["mask_2d"].numpy().astype(np.uint8), samples=stack(Xl), blocks=stack(Ml),
         blocks2=stack(M2l), meta=np.array([seed, 120, 10, 10, 1.0, p["lambd"], p["s"], p["delta_float"]]))

    # ---- (2) psgla + inpainting + TV(10) restated, non-square 1x3x24x40 ----------------
    x = ground_truth(3, 24, 40, seed=99)
    ns = reference_fidelity("inpainting", x, seed_ip=3)
    p = params["psgla_TV_defaults"]
    seed = 5
    tv = orc.TVDenoiser(n_it_max=10)
    Xl, Ml, M2l = run_psgla(ra, ns["init_torch"], ns["data_grad"], tv, 1.0, p["lambd"], p["s"],
                            p["delta_float"], 100, 10, 10, seed)
    save("psgla_inpaint_tv", x=x.numpy(), y=ns["y_t"].numpy(), init=ns["init_torch"].numpy(),
         mask2d=ns["mask_2d"].numpy().astype(np.uint8), samples=stack(Xl), blocks=stack(Ml),
         blocks2=stack(M2l), tv_x2=tv.x2.numpy(), tv_u2=tv.u2.numpy(),
         meta=np.array([seed, 100, 10, 10, 1.0, p["lambd"], p["s"], p["delta_float"], 10]))

    # ---- (3) psgla + deblurring (uniform and gaussian, l=4), clamp denoiser -----------
    for bt in ("uniform", "gaussian"):
        x = ground_truth(3, 32, 32, seed=7)
        ns = reference_fidelity("deblurring", x, blur_type=bt, si=1.0, l=4)
        p = params["psgla_DnCNN_defaults"]
        seed = 1
        Xl, Ml, M2l = run_psgla(ra, ns["init_torch"], ns["data_grad"], orc.ClampDenoiser(), 1.0,
                                p["lambd"], p["s"], p["delta_float"], 60, 10, 10, seed)
        save(f"psgla_deblur_{bt}", x=x.numpy(), y=ns["y_t"].numpy(), init=ns["init_torch"].numpy(),
             hcorr=ns["hcorr_torch"][0, 0].numpy(), samples=stack(Xl), blocks=stack(Ml),
             blocks2=stack(M2l),
             meta=np.array([seed, 60, 10, 10, 1.0, p["lambd"], p["s"], p["delta_float"], 4]))

    # ---- (4) pnpula + inpainting, prior from a clamp "denoiser" (prior_grad closure) ----
    x = ground_truth(3, 32, 32, seed=11)
    ns = reference_fidelity("inpainting", x)
    p = params["pnp_ula_DRUNet_N1e6"]
    s2t = torch.tensor(p["s1"] ** 2, dtype=torch.float32)
    alphat = torch.tensor(1.0, dtype=torch.float32)
    den = orc.ClampDenoiser()

    def prior_grad(xx):
        return alphat * (den.forward(xx, p["s1"]) - xx) / s2t
    seed = 2
    Xl, Ml, M2l = run_pnpula(ra, ns["init_torch"], ns["data_grad"], prior_grad,
                             torch.tensor(p["delta_float"], dtype=torch.float32),
                             torch.tensor(p["lambd"], dtype=torch.float32), 120, 10, 10, seed)
    save("pnpula_inpaint_clamp", x=x.numpy(), y=ns["y_t"].numpy(), init=ns["init_torch"].numpy(),
         mask2d=ns["mask_2d"].numpy().astype(np.uint8), samples=stack(Xl), blocks=stack(Ml),
         blocks2=stack(M2l), meta=np.array([seed, 120, 10, 10, 1.0, p["lambd"], p["s1"], p["delta_float"]]))

    # ---- (5) psgla, alpha=0.3, tiny fixed conv denoiser (pins the relaxation) ----------
    x = ground_truth(3, 16, 16, seed=21)
    ns = reference_fidelity("inpainting", x, seed_ip=4)
    g = torch.Generator().manual_seed(77)
    w = (torch.rand((3, 3, 3, 3), generator=g) - 0.5) * 0.1
    b = (torch.rand((3,), generator=g) - 0.5) * 0.01
    den = orc.TinyConvDenoiser(w, b)
    p = params["psgla_DnCNN_defaults"]
    seed = 9
    Xl, Ml, M2l = run_psgla(ra, ns["init_torch"], ns["data_grad"], den, 0.3, p["lambd"], p["s"],
                            p["delta_float"], 50, 5, 4, seed)
    save("psgla_inpaint_conv_alpha03", x=x.numpy(), y=ns["y_t"].numpy(), init=ns["init_torch"].numpy(),
         mask2d=ns["mask_2d"].numpy().astype(np.uint8), weight=w.numpy(), bias=b.numpy(),
         samples=stack(Xl), blocks=stack(Ml), blocks2=stack(M2l),
         meta=np.array([seed, 50, 5, 4, 0.3, p["lambd"], p["s"], p["delta_float"]]))

    # ---- (6) the inpainting mask of the 256x256 synthetic problem (CPU generator) -------
    x = ground_truth(3, 256, 256)
    ns = reference_fidelity("inpainting", x, seed_ip=0)
    save("mask_256_seed0", mask_bits=np.packbits(ns["mask_2d"].numpy().astype(np.uint8)))

    with open(os.path.join(HERE, "params.json"), "w") as f:
        json.dump(params, f, indent=1, sort_keys=True)
    print("wrote params.json")

    make_postproc()


def reference_postproc(im, samples_t, mmse_t, mmse2_t, y_t, init_torch, grayscale=False):
    """Execute the reference's per-image post-processing, sampling_images.py:371-442, on given
    chain outputs.  PSNR / ssim are bound to this build's metrics.psnr / metrics.ssim (scikit-image
    is not installed): the fixture pins everything AROUND them -- sample / block conversion, the
    running-MMSE curve (range(1, n)), MMSE, std, diff, min / max -- to the reference's own code."""
    from psgla_for_posterior_sampling_amd import metrics
    pars = types.SimpleNamespace(grayscale=grayscale)
    ns = dict(np=np, torch=torch, pars=pars, im=im, Samples_t=samples_t, Mmse_t=mmse_t, Mmse2_t=mmse2_t,
              y_t=y_t, init_torch=init_torch, PSNR=metrics.psnr, ssim=metrics.ssim)
    exec(compile(reference_source("sampling_images.py", 371, 442), "sampling_images.py:371", "exec"), ns)
    return ns


def make_postproc():
    """(7) sampling_images.py:371-442 on the chain outputs of fixture (2) (psgla + TV): the
    reference's result-dict values, for metrics.analyse_run (tests/test_metrics_cli.py)."""
    z = np.load(os.path.join(HERE, "psgla_inpaint_tv.npz"))
    im = np.float32(np.transpose(z["x"][0], (1, 2, 0)))
    samples_t = [torch.from_numpy(s) for s in z["samples"]]
    mmse_t = [torch.from_numpy(s) for s in z["blocks"]]
    mmse2_t = [torch.from_numpy(s) for s in z["blocks2"]]
    ns = reference_postproc(im, samples_t, mmse_t, mmse2_t, torch.from_numpy(z["y"]), torch.from_numpy(z["init"]))
    save("postproc_inpaint_tv", PSNR_sample=np.array(ns["Psnr_sample"], np.float64),
         SIM_sample=np.array(ns["SIM_sample"], np.float64), PSNR_mmse=np.array(ns["PSNR_list"], np.float64),
         SIM_list=np.array(ns["SIM_list"], np.float64), Min_sample=np.array(ns["Min_sample"]),
         Max_sample=np.array(ns["Max_sample"]), observation=ns["y"], init=ns["init"], PSNR_y=ns["psb"],
         SIM_y=ns["ssb"], MMSE=ns["xmmse"], PSNR_MMSE=ns["pmmse"], SIM_MMSE=ns["smmse"], std=ns["std"],
         diff=ns["diff"], mean_list=ns["mean_list"])


if __name__ == "__main__":
    if sys.argv[1:] == ["postproc"]:
        make_postproc()
    else:
        main()
