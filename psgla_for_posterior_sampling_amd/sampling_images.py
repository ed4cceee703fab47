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
  --allow_random_weights, --graph_steps, --batch_size, --tv_restart.

Batched and multi-GPU runs (build-specific; BASELINE configs 4-5 run CBSD68 over 8 GPUs).  Every image
is one Langevin chain whose noise is keyed by (--seed_alg, chain id); the chain id of image i is its rank
in the dataset listing stably sorted by image shape (= i for a dataset of one shape, e.g. set1c), so a
chain's samples do not depend on how images are batched or sharded.  ``--batch_size B`` groups the
images of one shape, in listing order, into batches of up to B chains that run as ONE psgla / pnpula
call ((B, C, H, W) state); under ``torch.distributed.run`` the image indices [indx_start, n) are split
contiguously over the ranks (one GPU per rank: cuda:(gpu_number + LOCAL_RANK)), each rank runs its
share, and rank 0 gathers every image's record and writes the reference's im_i/ directories.
TV warm start: the reference carries the TV prox state (x2, u2) from image k to image k+1
(sampling_images.py:138, reused in the :265 loop); that is kept for --batch_size 1 on one rank.  A
batched or sharded run starts the TV prox fresh for every image (x2 = Y, u2 = 0, as the reference
does for its first image); ``--tv_restart`` makes a sequential run do the same, which is the run a
batched one equals.  DnCNN / DRUNet have no state across images.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

from . import metrics
from .denoisers import DenoiserPrior, DnCNN, DRUNet, TVDenoiser
from .fidelity import BlurFidelity, InpaintingFidelity, deblurring_problem, inpainting_problem
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
    p.add_argument("--batch_size", type=int, default=1, help="chains (images of one shape) per psgla call")
    p.add_argument("--tv_restart", action="store_true", help="fresh TV prox state for every image")
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


PLUMBING_RESIDUAL_SCALE = 1e-3


@torch.no_grad()
def plumbing_residual_scale_(conv: torch.nn.Conv2d, scale: float = PLUMBING_RESIDUAL_SCALE) -> None:
    """A random-init DnCNN (no weights offline) stands in for the trained one in plumbing runs.  Raw, it is not a
    denoiser: its default-init layers shrink the signal, so out_conv(h) + x is x plus out_conv's bias, about
    ±0.04 per pixel and step, and the chain drifts without bound (PSNR_MMSE -21 dB after 1,000 steps).
    Scaling the residual branch's output layer by 1e-3 keeps D = id + a small bounded residual, so the chain stays
    on the observation's scale like a trained network's, and rounding differences between runs stay rounding."""
    conv.weight.mul_(scale)
    if conv.bias is not None:
        conv.bias.mul_(scale)


def make_denoiser(pars, device):
    if pars.den == "TV":
        return TVDenoiser(n_it_max=pars.den_TV_it)
    # random-init networks (--allow_random_weights, plumbing runs) are seeded: every rank of a sharded run
    # and every run of a comparison build the same network
    torch.manual_seed(pars.seed_alg)
    if pars.den == "DnCNN":
        w = os.path.join(pars.weights_dir, "dncnn_sigma2_lipschitz_color.pth")
        if not os.path.exists(w) and not pars.allow_random_weights:
            raise FileNotFoundError(f"{w} not found (DnCNN weights; --allow_random_weights for plumbing runs)")
        net = DnCNN(in_channels=3, out_channels=3, pretrained=w if os.path.exists(w) else None, device=device)
        if not os.path.exists(w):
            plumbing_residual_scale_(net.out_conv)
        return net
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


def _problem(pars, im: np.ndarray, device):
    """The inverse problem of one image (sampling_images.py:283-341), its generator seeded per image as in
    the reference: (data term, y_t (1, C, H, W), init (1, C, H, W), mask_2d or None, mask or None)."""
    if pars.grayscale:
        im_t = torch.from_numpy(np.ascontiguousarray(im)).float().unsqueeze(0).unsqueeze(0).to(device)
    else:
        im_t = torch.from_numpy(np.transpose(np.ascontiguousarray(im), (2, 0, 1))).float().unsqueeze(0).to(device)
    if pars.Pb == "inpainting":
        data_grad, y_t, init_torch, mask_2d, mask = inpainting_problem(im_t, seed_ip=pars.seed_ip, prop=pars.prop,
                                                                       sigma=pars.sigma)
        return data_grad, y_t, init_torch, mask_2d, mask
    if pars.Pb == "deblurring":
        data_grad, y_t, init_torch = deblurring_problem(im_t, seed_ip=pars.seed_ip, l=pars.l,
                                                        blur_type=pars.blur_type, si=pars.si, sigma=pars.sigma)
        return data_grad, y_t, init_torch, None, None
    raise ValueError("unknown --Pb " + pars.Pb)


def restore_batch(pars, argv, ims, chain0: int, denoiser, device):
    """The reference's per-image loop body (sampling_images.py:265-470) for len(ims) images of one shape
    run as ONE chain batch (chain ids chain0 ..): returns [(record, extras, mask)] per image.  With one
    image this is exactly the reference's run of that image."""
    N, s, lambd, delta, n_inter, ex = algorithm_parameters(pars, argv)
    n_inter_mmse = int(np.copy(n_inter))
    dtype = torch.float32
    alphat = torch.tensor(pars.alpha, dtype=dtype, device=device)
    probs = [_problem(pars, im, device) for im in ims]
    B = len(ims)
    y_b = torch.cat([p[1] for p in probs], dim=0).contiguous()
    init_b = torch.cat([p[2] for p in probs], dim=0).contiguous()
    if B == 1:
        data_grad = probs[0][0]
    elif pars.Pb == "inpainting":
        # one shape, one seed_ip: every image of the batch has the same mask (sampling_images.py:285-290)
        data_grad = InpaintingFidelity(probs[0][3], y_b, probs[0][0].sigma2)
    else:
        f0 = probs[0][0]
        data_grad = BlurFidelity(f0.hconv, f0.hcorr, f0.l, y_b, f0.sigma2t)
    name = "sigma{}_s{}".format(pars.sigma, int(255 * s))
    lambdt = torch.tensor(lambd, dtype=dtype, device=device)
    kw = dict(seed=pars.seed_alg, device=device, n_iter=N, n_inter=n_inter, n_inter_mmse=n_inter_mmse,
              path=pars._path_im, save_images_online=pars.save_images_online, name=name, chain0=chain0)
    if pars.graph_steps is not None:
        kw["graph_steps"] = pars.graph_steps
    if pars.alg == "psgla":
        Samples_t, Mmse_t, Mmse2_t = psgla(init=init_b, data_grad=data_grad, denoiser=denoiser, alpha=alphat,
                                           lambd=lambdt, sig_float=s, delta=delta, **kw)
    else:
        s1, s2t = ex["s1"], torch.tensor(ex["s2"], dtype=dtype, device=device)
        prior_grad = DenoiserPrior(denoiser, s1, alphat, s2t)    # alphat*(D(x, s1) - x)/s2t (:156-157)
        Samples_t, Mmse_t, Mmse2_t = pnpula(init=init_b, data_grad=data_grad, prior_grad=prior_grad,
                                            delta=torch.tensor(delta, dtype=dtype, device=device), lambd=lambdt,
                                            **kw)
    out = []
    for b, im in enumerate(ims):
        pick = (lambda lst: [t[b] for t in lst]) if B > 1 else (lambda lst: lst)   # noqa: E731
        record, extras = metrics.analyse_run(im, pick(Samples_t), pick(Mmse_t), pick(Mmse2_t), probs[b][1],
                                             probs[b][2], pars.grayscale)
        record.update({"n_iter": N, "s": s, "alpha": pars.alpha, "c_min": 0, "c_max": 1, "sigma": pars.sigma,
                       "l": pars.l, "lambda": lambd, "delta": delta})
        out.append((record, extras, probs[b][4], name))
    return out


def restore_image(pars, argv, im: np.ndarray, denoiser, device, path_result_im: str, chain: int = 0):
    """One image of the reference's loop (sampling_images.py:265-529), results written to path_result_im."""
    pars._path_im = path_result_im
    record, extras, mask, name = restore_batch(pars, argv, [im], chain, denoiser, device)[0]
    write_result(pars, path_result_im, name, record, mask)
    return record, extras


def write_result(pars, path_result_im: str, name: str, record: dict, mask):
    """sampling_images.py:470 (the result dict) and the images of :523-535."""
    os.makedirs(path_result_im, exist_ok=True)
    np.save(path_result_im + "/" + name + "_result.npy", record)
    if not pars.no_plots:
        _save_images(pars, path_result_im, name, record, mask)
    print("The output PSNR : {:.2f} dB / output SSIM : {:.2f}".format(record["PSNR_MMSE"], record["SIM_MMSE"]))


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


def dataset_files(pars):
    input_path = os.path.join(pars.datasets_root, pars.dataset_name)
    return [os.path.join(input_path, f) for f in sorted(os.listdir(input_path))]


def image_shape(path: str):
    from PIL import Image
    with Image.open(path) as im:
        return im.size[::-1]


def chain_ids(files):
    """Chain id of every image: its rank in the listing stably sorted by image shape (module docstring)."""
    order = sorted(range(len(files)), key=lambda i: (image_shape(files[i]), i))
    ids = [0] * len(files)
    for r, i in enumerate(order):
        ids[i] = r
    return ids


def shape_batches(indices, files, ids, batch_size: int):
    """Batches of up to batch_size images of one shape with consecutive chain ids, in listing order of
    their first image."""
    groups = {}
    for i in indices:
        groups.setdefault(image_shape(files[i]), []).append(i)
    batches = []
    for g in groups.values():
        cur = []
        for i in g:
            if cur and (len(cur) == batch_size or ids[i] != ids[cur[-1]] + 1):
                batches.append(cur)
                cur = []
            cur.append(i)
        if cur:
            batches.append(cur)
    return sorted(batches, key=lambda b: b[0])


def load_image(pars, path: str) -> np.ndarray:
    im_int = read_image(path)
    im = np.float32(im_int / 255.)
    if pars.grayscale:
        im = np.float32(im_int[..., 0] / 255.)
    return im


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    pars = build_parser().parse_args(argv)
    if pars.alg not in ("psgla", "pnp_ula"):
        raise NotImplementedError(f"--alg {pars.alg}: only psgla and pnp_ula are part of this build")
    if pars.batch_size < 1:
        raise ValueError("--batch_size must be >= 1")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(torch.cuda.device_count(), 1)
    device = torch.device("cuda:" + str((pars.gpu_number + local) % ndev))
    obj_group = None
    if world > 1:
        # no collective on the hot path: the per-image results are gathered once at the end -- their arrays over
        # RCCL (device tensors) when every rank has a GPU of its own, the small metadata over a gloo group
        import torch.distributed as dist
        from .sharding import dist_backend
        backend = dist_backend(int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
        if backend == "nccl":
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=device)
            obj_group = dist.new_group(backend="gloo")
        else:
            dist.init_process_group(backend)
    sequential = world == 1 and pars.batch_size == 1
    if pars.save_images_online and not sequential:
        raise ValueError("--save_images_online needs a sequential run (--batch_size 1, one rank)")
    path_result = result_path(pars, argv) if rank == 0 else None
    if world > 1:
        dist.barrier()
        path_result = result_path(pars, argv)
    files = dataset_files(pars)
    ids = chain_ids(files)
    indices = list(range(pars.indx_start, len(files)))
    denoiser = make_denoiser(pars, device)   # one object for the whole dataset, as the reference (:138)
    if sequential:
        records = []
        for i in indices:
            path_result_im = os.path.join(path_result, "im_" + str(i))
            os.makedirs(path_result_im, exist_ok=True)
            if pars.tv_restart and isinstance(denoiser, TVDenoiser):
                denoiser.restart = True
            records.append(restore_image(pars, argv, load_image(pars, files[i]), denoiser, device, path_result_im,
                                         chain=ids[i])[0])
        return records
    from .sharding import chain_range
    a, b = chain_range(len(indices), world, rank)
    mine = indices[a:b]
    local_out = {}
    pars._path_im = ""
    for batch in shape_batches(mine, files, ids, pars.batch_size):
        if isinstance(denoiser, TVDenoiser):
            denoiser.restart = True              # batched / sharded: fresh TV state for every image
        ims = [load_image(pars, files[i]) for i in batch]
        for i, (record, _extras, mask, name) in zip(batch, restore_batch(pars, argv, ims, ids[batch[0]], denoiser,
                                                                           device)):
            local_out[i] = (record, None if mask is None else mask.cpu(), name)
    from .sharding import gather_records, reduce_dataset_psnr
    psnr_sum, ssim_sum, n_img = reduce_dataset_psnr(local_out, world, device)
    gathered = gather_records(local_out, world, rank, device, obj_group)
    records = []
    if rank == 0:
        for i in indices:
            record, mask, name = gathered[i]
            write_result(pars, os.path.join(path_result, "im_" + str(i)), name, record, mask)
            records.append(record)
        # not in the reference's output: only for the runs it has no counterpart of (batched or sharded)
        if n_img and (world > 1 or getattr(pars, "batch_size", 1) > 1):
            print("Dataset ({} images): mean output PSNR {:.2f} dB / mean output SSIM {:.2f}".format(
                n_img, psnr_sum / n_img, ssim_sum / n_img))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return records


if __name__ == "__main__":
    main()
