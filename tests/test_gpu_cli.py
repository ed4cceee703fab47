"""End-to-end CLI run (sampling_images.py surface) on a tiny synthetic dataset, on the GPU."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dataset(root, n=2, h=32, w=48):
    from PIL import Image
    d = os.path.join(root, "datasets", "synth")
    os.makedirs(d)
    rng = np.random.default_rng(5)
    for i in range(n):
        yy, xx = np.mgrid[0:h, 0:w]
        im = np.stack([(xx * 5 + 40 * i) % 256, (yy * 7) % 256, ((xx + yy) * 3) % 256], axis=2)
        im = np.clip(im + rng.integers(0, 10, im.shape), 0, 255).astype(np.uint8)
        Image.fromarray(im).save(os.path.join(d, f"{i:04d}.png"))
    return os.path.join(root, "datasets")


def test_cli_psgla_tv_inpainting(tmp_path):
    from psgla_for_posterior_sampling_amd import metrics
    from psgla_for_posterior_sampling_amd import sampling_images as SI
    droot = _dataset(str(tmp_path))
    argv = ["--alg", "psgla", "--den", "TV", "--Pb", "inpainting", "--dataset_name", "synth",
            "--datasets_root", droot, "--results_root", str(tmp_path / "results"), "--no_plots"]
    recs = SI.main(argv)
    assert len(recs) == 2
    base = os.path.join(str(tmp_path / "results"), "images", "inpainting", "synth", "psgla", "TV")
    for i, r in enumerate(recs):
        files = os.listdir(os.path.join(base, f"im_{i}"))
        res = [x for x in files if x.endswith("_result.npy")]
        assert len(res) == 1
        d = np.load(os.path.join(base, f"im_{i}", res[0]), allow_pickle=True).item()   # our own output file
        assert d["n_iter"] == 1000 and abs(d["lambda"] - 10.0) < 1e-12
        assert len(d["PSNR_sample"]) == 100 and len(d["PSNR_mmse"]) == 90 - 1
        assert np.isfinite(d["PSNR_MMSE"]) and d["PSNR_MMSE"] > d["PSNR_y"]
        assert abs(d["PSNR_MMSE"] - metrics.psnr(d["ground_truth"], d["MMSE"])) < 1e-9


def test_cli_pnpula_deblurring_random_dncnn(tmp_path):
    from psgla_for_posterior_sampling_amd import sampling_images as SI
    droot = _dataset(str(tmp_path), n=1)
    argv = ["--alg", "pnp_ula", "--den", "DnCNN", "--Pb", "deblurring", "--dataset_name", "synth", "--N", "1000",
            "--datasets_root", droot, "--results_root", str(tmp_path / "results"), "--no_plots",
            "--allow_random_weights", "--weights_dir", str(tmp_path / "none")]
    recs = SI.main(argv)
    assert len(recs) == 1 and np.isfinite(recs[0]["PSNR_y"])
    assert len(recs[0]["PSNR_sample"]) == 1000    # n_inter = int(N / 1000) = 1: every step stored


def test_cli_psgla_inpainting_random_dncnn(tmp_path):
    """Config 3's command (--den DnCNN, random-init weights offline): the DenoiserChains path."""
    from psgla_for_posterior_sampling_amd import sampling_images as SI
    droot = _dataset(str(tmp_path), n=1)
    argv = ["--alg", "psgla", "--den", "DnCNN", "--Pb", "inpainting", "--dataset_name", "synth", "--N", "1000",
            "--datasets_root", droot, "--results_root", str(tmp_path / "results"), "--no_plots",
            "--allow_random_weights", "--weights_dir", str(tmp_path / "none"), "--graph_steps", "20"]
    recs = SI.main(argv)
    assert len(recs) == 1 and np.isfinite(recs[0]["PSNR_MMSE"])
    assert len(recs[0]["PSNR_sample"]) == 1000


def test_cli_pnpula_inpainting_random_drunet(tmp_path):
    """Config 5's command shape (--alg pnp_ula --den DRUNet): UlaChains with a DenoiserPrior."""
    from psgla_for_posterior_sampling_amd import sampling_images as SI
    droot = _dataset(str(tmp_path), n=1)
    argv = ["--alg", "pnp_ula", "--den", "DRUNet", "--Pb", "inpainting", "--dataset_name", "synth", "--N", "1000",
            "--s", "5", "--datasets_root", droot, "--results_root", str(tmp_path / "results"), "--no_plots",
            "--allow_random_weights", "--weights_dir", str(tmp_path / "none"), "--graph_steps", "20"]
    recs = SI.main(argv)
    assert len(recs) == 1 and np.isfinite(recs[0]["PSNR_y"])
    assert len(recs[0]["PSNR_sample"]) == 1000


def test_bench_multirank_rehearsal():
    """bench.py's multi-rank path (torch.distributed.run, strong split of the 64 chains, barriers, max over
    ranks, the PSNR all_reduce) with 2 ranks on this box's one GPU over gloo (PSGLA_DIST_BACKEND): every
    chain's samples do not depend on the split, so the mean MMSE PSNR equals the 1-rank run's."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = ["bench.py", "--steps", "20", "--warmup", "5", "--no-cpu", "--kernel-iters", "3", "--warmup-seconds", "0"]
    env = dict(os.environ, PSGLA_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", "29533"] + base + ["--gpus", "2"],
                         cwd=repo, env=env, capture_output=True, text=True, timeout=240)
    assert two.returncode == 0, two.stderr[-2000:]
    d2 = json.loads([l for l in two.stdout.splitlines() if l.startswith("{")][-1])
    one = subprocess.run([sys.executable] + base, cwd=repo, capture_output=True, text=True, timeout=240)
    assert one.returncode == 0, one.stderr[-2000:]
    d1 = json.loads([l for l in one.stdout.splitlines() if l.startswith("{")][-1])
    assert d2["n_gpus"] == 2 and d2["config"]["chains_per_gpu"] == 32 and d2["config"]["global_batch"] == 64
    assert d2["scaling"] == "strong" and d2["value"] > 0
    assert abs(d2["mmse_psnr_mean_db"] - d1["mmse_psnr_mean_db"]) < 1e-9
