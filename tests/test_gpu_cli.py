"""End-to-end CLI run (sampling_images.py surface) on a tiny synthetic dataset, on the GPU."""
import os
import socket

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
    base = ["bench.py", "--steps", "20", "--warmup", "5", "--no-cpu", "--warmup-seconds", "0"]
    env = dict(os.environ, PSGLA_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port)] + base + ["--gpus", "2"],
                         cwd=repo, env=env, capture_output=True, text=True, timeout=240)
    assert two.returncode == 0, two.stderr[-2000:]
    d2 = json.loads([l for l in two.stdout.splitlines() if l.startswith("{")][-1])
    one = subprocess.run([sys.executable] + base, cwd=repo, capture_output=True, text=True, timeout=240)
    assert one.returncode == 0, one.stderr[-2000:]
    d1 = json.loads([l for l in one.stdout.splitlines() if l.startswith("{")][-1])
    assert d2["n_gpus"] == 2 and d2["config"]["chains_per_gpu"] == 32 and d2["config"]["global_batch"] == 64
    assert d2["scaling"] == "strong" and d2["value"] > 0
    assert abs(d2["mmse_psnr_mean_db"] - d1["mmse_psnr_mean_db"]) < 1e-9
    # the N > 1 line names every rank's device and PCI address (one GPU here: both ranks on it)
    pl = d2["config"]["placement"]
    assert [p["rank"] for p in pl] == [0, 1] and [p["chains"] for p in pl] == [[0, 32], [32, 64]]
    assert d2["config"]["distinct_gpus"] == len({p["pci"] for p in pl}) == 1


def _two_shape_dataset(root):
    """5 images, two shapes interleaved: 24x32 (indices 0, 1, 3) and 32x24 (2, 4)."""
    from PIL import Image
    d = os.path.join(root, "datasets", "mixed")
    os.makedirs(d)
    rng = np.random.default_rng(11)
    for i, (h, w) in enumerate([(24, 32), (24, 32), (32, 24), (24, 32), (32, 24)]):
        im = rng.integers(0, 256, (h, w, 3)).astype(np.uint8)
        Image.fromarray(im).save(os.path.join(d, f"{i:04d}.png"))
    return os.path.join(root, "datasets")


def _records(root, n):
    """Every image's result dict under a results root (the CLI's path scheme adds the typed flags)."""
    base = next(d for d, subs, _ in os.walk(root) if "im_0" in subs)
    out = []
    for i in range(n):
        res = [x for x in os.listdir(os.path.join(base, f"im_{i}")) if x.endswith("_result.npy")]
        assert len(res) == 1
        out.append(np.load(os.path.join(base, f"im_{i}", res[0]), allow_pickle=True).item())   # our own file
    return out


def _same_records(a, b, exact):
    for ra, rb in zip(a, b):
        for k in ("observation", "init"):
            np.testing.assert_array_equal(np.asarray(ra[k]), np.asarray(rb[k]), err_msg=k)
        for k in ("PSNR_sample", "PSNR_mmse", "SIM_sample", "MMSE", "std"):
            if exact:
                np.testing.assert_array_equal(np.asarray(ra[k]), np.asarray(rb[k]), err_msg=k)
            else:
                # measured on the bounded plumbing chain (profiles/r06b_cli_dncnn.log): MMSE <= 1.4e-5 relative
                # (1e-5 absolute floor in the denominator), std <= 5.5e-7; the bounds leave a 7x margin
                tol = dict(rtol=1e-4, atol=1e-5)
                np.testing.assert_allclose(np.asarray(ra[k]), np.asarray(rb[k]), err_msg=k, **tol)
        assert (ra["PSNR_MMSE"] == rb["PSNR_MMSE"]) if exact else abs(ra["PSNR_MMSE"] - rb["PSNR_MMSE"]) < 1e-3


@pytest.mark.parametrize("den", ["DnCNN", "TV"])
def test_cli_batched_and_sharded_equal_sequential(tmp_path, den):
    """The CLI over a two-shape dataset: sequential (--batch_size 1, the reference's loop), batched
    (--batch_size 4: one psgla call per shape group) and sharded over 2 ranks (torch.distributed.run, gloo,
    both on this box's GPU) write the same per-image records.  Chain ids follow the shape-sorted listing,
    so every image's noise is the same in all three runs; TV starts fresh for every image in the batched
    runs, and --tv_restart makes the sequential run do the same: bit-identical records.  DnCNN: identical
    to fp32 rounding (MIOpen picks its convolution solver per batch size)."""
    import subprocess
    import sys
    from psgla_for_posterior_sampling_amd import sampling_images as SI
    droot = _two_shape_dataset(str(tmp_path))
    files = SI.dataset_files(SI.build_parser().parse_args(["--dataset_name", "mixed", "--datasets_root", droot]))
    assert SI.chain_ids(files) == [0, 1, 3, 2, 4]
    common = ["--alg", "psgla", "--den", den, "--Pb", "inpainting", "--dataset_name", "mixed", "--N", "1000",
              "--datasets_root", droot, "--no_plots", "--allow_random_weights", "--weights_dir", str(tmp_path / "w"),
              "--graph_steps", "20"]
    if den == "TV":
        common += ["--tv_restart"]
    runs = {}
    for tag, extra in (("seq", ["--batch_size", "1"]), ("batch", ["--batch_size", "4"])):
        SI.main(common + ["--results_root", str(tmp_path / tag)] + extra)
        runs[tag] = _records(str(tmp_path / tag), 5)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=repo)
    env.pop("PSGLA_DIST_BACKEND", None)   # the CLI's own choice: gloo here (two ranks, one GPU), nccl on a node
    sock = socket.socket()                # a free port, not a fixed one a leftover rendezvous may still hold
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), "-m",
                          "psgla_for_posterior_sampling_amd.sampling_images"] + common
                         + ["--results_root", str(tmp_path / "ranks"), "--batch_size", "4"],
                         cwd=repo, env=env, capture_output=True, text=True, timeout=300)
    assert two.returncode == 0, two.stderr[-3000:]
    assert "Dataset (5 images): mean output PSNR" in two.stdout, two.stdout[-2000:]
    runs["ranks"] = _records(str(tmp_path / "ranks"), 5)
    # the comparison is only meaningful on a bounded chain (a raw random DnCNN drifted to MMSE values of
    # -23 .. 13 and amplified the conv rounding; the CLI's plumbing network is D = id + 1e-3 x residual)
    for r in runs["seq"]:
        assert np.abs(np.asarray(r["MMSE"])).max() < 2.0 and r["PSNR_MMSE"] > r["PSNR_y"] - 3.0, r["PSNR_MMSE"]
    if den != "TV":
        for tag in ("batch", "ranks"):
            for k in ("MMSE", "std"):
                d = max(float(np.max(np.abs(np.asarray(ra[k]) - np.asarray(rb[k])) / (np.abs(np.asarray(rb[k])) + 1e-5)))
                        for ra, rb in zip(runs[tag], runs["seq"]))
                print(f"DnCNN {tag} vs seq: max rel diff of {k} = {d:.3g}")
    # TV (the HIP step alone) is bit-identical; DnCNN's forward runs on MIOpen, whose convolution solver is
    # chosen per batch size (B = 1, 2, 3 here), so its records agree to fp32 rounding
    _same_records(runs["batch"], runs["seq"], exact=den == "TV")
    _same_records(runs["ranks"], runs["seq"], exact=den == "TV")


@pytest.mark.parametrize("batch", [1])
def test_cli_castle_known_answer(tmp_path, batch):
    """The one published number reachable offline (no weights): PSGLA + TV on set1c's castle (481 x 321),
    inpainting 50 %, sigma = 1/255, the CLI defaults for --den TV (N = 1000, s = 10/255, lambda = 10).
    The reference's Figure 2 reports 28.09 dB (README.md:14-15); its own psgla driven by the TV restatement
    gives 28.23 dB on the CPU-generator mask.  The mask here comes from the ROCm generator
    (the reference's from CUDA's), so this is a tolerance check: PSNR_MMSE within 0.3 dB of both, the
    observation's PSNR ~8.7 dB.  tests/golden/set1c/castle.png is the reference's dataset image (data)."""
    from psgla_for_posterior_sampling_amd import sampling_images as SI
    droot = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    argv = ["--alg", "psgla", "--den", "TV", "--dataset_name", "set1c", "--datasets_root", droot,
            "--results_root", str(tmp_path / "results"), "--no_plots", "--batch_size", str(batch)]
    recs = SI.main(argv)
    assert len(recs) == 1
    r = recs[0]
    assert r["n_iter"] == 1000 and r["MMSE"].shape == (481, 321, 3)
    assert abs(r["PSNR_y"] - 8.73) < 0.1, r["PSNR_y"]
    assert abs(r["PSNR_MMSE"] - 28.23) < 0.3 and abs(r["PSNR_MMSE"] - 28.09) < 0.3, r["PSNR_MMSE"]
