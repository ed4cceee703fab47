"""Command-line driver with the reference's ``sampling_images.py`` surface (sampling_images.py:19-46).

    python -m psgla_for_posterior_sampling_amd.sampling_images --alg psgla --den TV --Pb inpainting \
        --dataset_name set1c [--N 10000] ...

Same flags, defaults and *flag-presence* semantics (a flag typed on the command line changes
the parameter choice and the result path even when its value equals the default,
sampling_images.py:52-94, :147-198), the same result directory scheme, result dictionary
(np.save of a dict, sampling_images.py:441-466) and output images.  The Langevin loop runs on
the MI355X path (psgla / pnpula of this package); the per-image post-processing (PSNR / SSIM per
sample and of the running MMSE, std, ...) is metrics.analyse_run.

Differences, all outside the hot path:
* --alg pnp / red / diffpir / baseline are not part of this build (NotImplementedError);
* --den GSDRUNet / Prox_DRUNet are not available (no deepinv, no weights); DnCNN and DRUNet
  (architectures restated in denoisers.py) load deepinv-format weights from --weights_dir
  (``--allow_random_weights`` runs random-init networks for plumbing tests);
* extra flags: --datasets_root, --weights_dir, --results_root, --no_plots,
  --allow_random_weights, --graph_steps.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

from . import metrics
from .denoisers import DenoiserPrior, DnCNN, DRUNet, TVDenoiser
from .fidelity import deblurring_problem, inpainting_problem
from .restoration_algorithms import pnpula, psgla


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser()
    p.add_argument("--N", type=int, default=10000, help="number of iteration")
    p.add_argument("--alpha", type=float, default=1., help="relaxation parameter of the denoiser")
    p.add_argument("--s", type=float, default=5., help="denoiser parameter")
    p.add_argument("--dataset_name", type=str, default="set1c", help="dataset of images to reconstruct")
    p.add_argument("--path_result", type=str, default="images", help="results are saved in results/path_result")
    p.add_argument("--gpu_number", type=int, default=0, help="gpu number use")
    p.add_argument("--blur_type", type=str, default="uniform", help="uniform or gaussian blur")
    p.add_argument("--sigma", type=float, default=1., help="noise level of the observation")
    p.add_argument("--l", type=int, default=4, help="(2*l+1)*(2*l+1) is the size of the blur kernel")
    p.add_argument("--si", type=float, default=1., help="variance of the blur kernel (gaussian blur)")
    p.add_argument("--prop", type=float, default=0.5, help="proportion of masked pixels in random inpainting")
    p.add_argument("--delta", type=float, default=3e-5, help="step-size for the data-fidelity")
    p.add_argument("--lambd", type=float, default=1., help="regularization weights")
    p.add_argument("--zeta", type=float, default=0.8, help="regularization weights for DiffPIR")
    p.add_argument("--t_start", type=int, default=200, help="time of start for DiffPIR")
    p.add_argument("--seed_ip", type=int, default=0, help="seed for the inverse problem")
    p.add_argument("--seed_alg", type=int, default=0, help="seed for the algorithm running")
    p.add_argument("--Pb", type=str, default="inpainting", help="'deblurring' or 'inpainting'")
    p.add_argument("--grayscale", dest="grayscale", action="store_true")
    p.set_defaults(grayscale=False)
    p.add_argument("--save_images_online", dest="save_images_online", action="store_true")
    p.set_defaults(save_images_online=False)
    p.add_argument("--alg", type=str, default="psgla", help="'psgla' or 'pnp_ula'")
    p.add_argument("--den", type=str, default="DnCNN", help="'DnCNN' or 'TV'")
    p.add_argument("--den_TV_it", type=int, default=10, help="inner iterations of the TV prox per step")
    p.add_argument("--indx_start", type=int, default=0, help="index of the first image of the dataset")
    # build-specific
    p.add_argument("--datasets_root", type=str, default="datasets")
    p.add_argument("--weights_dir", type=str, default="Pretrained_models")
    p.add_argument("--results_root", type=str, default="results")
    p.add_argument("--no_plots", action="store_true")
    p.add_argument("--allow_random_weights", action="store_true")
    p.add_argument("--graph_steps", type=int, default=None)
    return p


def result_path(pars, argv) -> str:
    """sampling_images.py:52-94 (directories created along the way)."""
    given = lambda f: f in argv  # noqa: E731  flag-presence semantics of the reference
    path = os.path.join(pars.results_root, pars.path_result, pars.Pb)
    if given("--prop"):
        path = os.path.join(path, "prop_" + str(pars.prop))
    path = os.path.join(path, pars.dataset_name, pars.alg, pars.den)
    for flag, name in (("--s", "s"), ("--delta", "delta"), ("--lambd", "lambd"), ("--alpha", "alpha"),
                       ("--N", "N"), ("--seed_alg", "seed_alg"), ("--zeta", "zeta"), ("--t_start", "t_start"),
                       ("--den_TV_it", "den_TV_it")):
        if given(flag):
            path = os.path.join(path, name + "_" + str(getattr(pars, name)))
    os.makedirs(path, exist_ok=True)
    return path


def algorithm_parameters(pars, argv):
    """sampling_images.py:100-123 and :147-198: (N, s, lambd, delta, n_inter, extras)."""
    given = lambda f: f in argv  # noqa: E731
    sigma1 = pars.sigma / 255.0
    sigma2 = sigma1 ** 2
    alpha = pars.alpha
    N = pars.N
    if pars.alg == "pnp_ula":
        s = 2.0 / 255. if (not given("--s") and pars.den == "DnCNN") else pars.s
        s1 = s / 255.
        s2 = s1 ** 2
        N = 100000 if (not given("--N") and pars.den == "DnCNN") else pars.N
        lambd = 0.5 / (2 / sigma2 + alpha / s2)
        delta = 1 / 3 / (1 / sigma2 + 1 / lambd + alpha / s2)
        extras = {"s1": s1, "s2": s2}
    elif pars.alg == "psgla":
        if pars.den == "DnCNN":
            s = 2.0 / 255. if not given("--s") else pars.s / 255.
            lambd = 5.0 if not given("--lambd") else pars.lambd
        elif pars.den == "TV":
            s = 10.0 / 255. if not given("--s") else pars.s / 255.
            lambd = 10.0 if not given("--lambd") else pars.lambd
            N = 1000 if not given("--N") else pars.N
        else:
            s = pars.s / 255.
            lambd = pars.lambd
            N = pars.N
        delta = s ** 2
        extras = {}
    else:
        raise NotImplementedError(f"--alg {pars.alg}: only psgla and pnp_ula are part of this build "
                                  "(DESIGN.md section 8)")
    # n_inter is derived from pars.N, not from the overridden N (sampling_images.py:105)
    n_inter = int(pars.N / 1000)
    return N, s, lambd, delta, n_inter, extras


def make_denoiser(pars, device):
    if pars.den == "TV":
        return TVDenoiser(n_it_max=pars.den_TV_it)
    if pars.den == "DnCNN":
        w = os.path.join(pars.weights_dir, "dncnn_sigma2_lipschitz_color.pth")
        if not os.path.exists(w) and not pars.allow_random_weights:
            raise FileNotFoundError(f"{w} not found (DnCNN weights; --allow_random_weights for plumbing runs)")
        return DnCNN(in_channels=3, out_channels=3, pretrained=w if os.path.exists(w) else None, device=device)
    if pars.den == "DRUNet":
        w = os.path.join(pars.weights_dir, "drunet_color.pth")
        if not os.path.exists(w) and not pars.allow_random_weights:
            raise FileNotFoundError(f"{w} not found (DRUNet weights; --allow_random_weights for plumbing runs)")
        return DRUNet(in_channels=3, out_channels=3, pretrained=w if os.path.exists(w) else None, device=device)
    raise ValueError("Denoiser not implemented in this build: " + pars.den)


def read_image(path: str) -> np.ndarray:
    """utils_images.imread_uint (RGB uint8, gray expanded to 3 channels)."""
    from PIL import Image
    im = np.asarray(Image.open(path))
    if im.ndim == 2:
        im = np.stack([im] * 3, axis=2)
    return im[..., :3]


def restore_image(pars, argv, im: np.ndarray, denoiser, device, path_result_im: str):
    """One image of the reference's loop (sampling_images.py:265-529)."""
    N, s, lambd, delta, n_inter, ex = algorithm_parameters(pars, argv)
    n_inter_mmse = int(np.copy(n_inter))
    dtype = torch.float32
    alphat = torch.tensor(pars.alpha, dtype=dtype, device=device)
    if pars.grayscale:
        im_t = torch.from_numpy(np.ascontiguousarray(im)).float().unsqueeze(0).unsqueeze(0).to(device)
    else:
        im_t = torch.from_numpy(np.transpose(np.ascontiguousarray(im), (2, 0, 1))).float().unsqueeze(0).to(device)
    mask = None
    if pars.Pb == "inpainting":
        data_grad, y_t, init_torch, mask_2d, mask = inpainting_problem(im_t, seed_ip=pars.seed_ip, prop=pars.prop,
                                                                       sigma=pars.sigma)
    elif pars.Pb == "deblurring":
        data_grad, y_t, init_torch = deblurring_problem(im_t, seed_ip=pars.seed_ip, l=pars.l,
                                                        blur_type=pars.blur_type, si=pars.si, sigma=pars.sigma)
    else:
        raise ValueError("unknown --Pb " + pars.Pb)
    name = "sigma{}_s{}".format(pars.sigma, int(255 * s))
    lambdt = torch.tensor(lambd, dtype=dtype, device=device)
    kw = dict(seed=pars.seed_alg, device=device, n_iter=N, n_inter=n_inter, n_inter_mmse=n_inter_mmse,
              path=path_result_im, save_images_online=pars.save_images_online, name=name)
    if pars.alg == "psgla":
        if pars.graph_steps is not None:
            kw["graph_steps"] = pars.graph_steps
        Samples_t, Mmse_t, Mmse2_t = psgla(init=init_torch, data_grad=data_grad, denoiser=denoiser, alpha=alphat,
                                           lambd=lambdt, sig_float=s, delta=delta, **kw)
    else:
        s1, s2t = ex["s1"], torch.tensor(ex["s2"], dtype=dtype, device=device)
        prior_grad = DenoiserPrior(denoiser, s1, alphat, s2t)    # alphat*(D(x, s1) - x)/s2t (:156-157)
        if pars.graph_steps is not None:
            kw["graph_steps"] = pars.graph_steps
        Samples_t, Mmse_t, Mmse2_t = pnpula(init=init_torch, data_grad=data_grad, prior_grad=prior_grad,
                                            delta=torch.tensor(delta, dtype=dtype, device=device), lambd=lambdt,
                                            **kw)
    record, extras = metrics.analyse_run(im, Samples_t, Mmse_t, Mmse2_t, y_t, init_torch, pars.grayscale)
    record.update({"n_iter": N, "s": s, "alpha": pars.alpha, "c_min": 0, "c_max": 1, "sigma": pars.sigma,
                   "l": pars.l, "lambda": lambd, "delta": delta})
    np.save(path_result_im + "/" + name + "_result.npy", record)
    if not pars.no_plots:
        _save_images(pars, path_result_im, name, record, mask)
    print("The output PSNR : {:.2f} dB / output SSIM : {:.2f}".format(record["PSNR_MMSE"], record["SIM_MMSE"]))
    return record, extras


def _save_images(pars, path, name, rec, mask):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    cmap = "gray" if pars.grayscale else None
    plt.imsave(path + "/observation.png", np.clip(rec["observation"], 0, 1), cmap=cmap)
    plt.imsave(path + "/ground_truth.png", np.clip(rec["ground_truth"], 0, 1), cmap=cmap)
    plt.imsave(path + "/init.png", np.clip(rec["init"], 0, 1), cmap=cmap)
    plt.imsave(path + "/mmse_" + name + "_psnr{:.2f}_ssim{:.2f}.png".format(rec["PSNR_MMSE"], rec["SIM_MMSE"]),
               np.clip(rec["MMSE"], 0, 1), cmap=cmap)
    if pars.Pb == "inpainting" and mask is not None:
        m = np.transpose(mask.cpu().numpy()[0], (1, 2, 0))
        plt.imsave(path + "/error.png", np.clip(m * (rec["MMSE"] - rec["ground_truth"]), 0, 1), cmap=cmap)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    pars = build_parser().parse_args(argv)
    if pars.alg not in ("psgla", "pnp_ula"):
        raise NotImplementedError(f"--alg {pars.alg}: only psgla and pnp_ula are part of this build")
    device = torch.device("cuda:" + str(pars.gpu_number))
    path_result = result_path(pars, argv)
    denoiser = make_denoiser(pars, device)   # one object for the whole dataset, as the reference (:138)
    input_path = os.path.join(pars.datasets_root, pars.dataset_name)
    files = sorted(os.listdir(input_path))
    records = []
    for i in range(pars.indx_start, len(files)):
        path_result_im = os.path.join(path_result, "im_" + str(i))
        os.makedirs(path_result_im, exist_ok=True)
        im_int = read_image(os.path.join(input_path, files[i]))
        im = np.float32(im_int / 255.)
        if pars.grayscale:
            im = np.float32(im_int[..., 0] / 255.)
        records.append(restore_image(pars, argv, im, denoiser, device, path_result_im)[0])
    return records


if __name__ == "__main__":
    main()
