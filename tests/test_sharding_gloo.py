"""Multi-process sharding of chains (world size 2, gloo on CPU, 127.0.0.1).

The GPU path shards chains contiguously over ranks (sharding.chain_range) and keys each chain's
noise by its GLOBAL id, so the union of the ranks' chains equals the single-process run; the only
collectives are the final all_reduce of PSNR sums and all_gather of per-chain images
(sharding.reduce_psnr / gather_chains).  Each rank here runs the CPU checker
(oracle.psgla, one chain at a time, as the reference runs one chain per image) on its shard.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from psgla_for_posterior_sampling_amd.sharding import chain_range, gather_chains, psnr, reduce_psnr


def test_chain_range_partitions():
    for total in (0, 1, 5, 64, 65):
        for world in (1, 2, 3, 8):
            got = [chain_range(total, world, r) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == total
            for (a0, a1), (b0, b1) in zip(got, got[1:]):
                assert a1 == b0
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        chain_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


TOTAL = 5          # uneven split: 3 + 2
H = W = 8
N_ITER, N_INTER = 20, 5


def _run_chains(c0, c1):
    """Per-chain oracle runs: ground truth, blocks (nb, B, C, H, W) and last samples."""
    from oracle import psgla_oracle as orc
    gts, blocks, lasts = [], [], []
    for c in range(c0, c1):
        g = torch.Generator().manual_seed(1234 + c)
        x = torch.rand((1, 3, H, W), generator=g)
        dg, y, init, _ = orc.inpainting_problem(x, seed_ip=0)
        s = 10 / 255.0
        Xl, M, _ = orc.psgla(init, dg, orc.ClampDenoiser(), torch.tensor(1.0), torch.tensor(10.0), sig_float=s,
                             delta=s ** 2, n_iter=N_ITER, n_inter=N_INTER, n_inter_mmse=N_INTER - 1, seed=0, chain=c)
        gts.append(x[0])
        blocks.append(torch.stack(M))
        lasts.append(Xl[-1])
    if not gts:
        return torch.zeros((0, 3, H, W)), torch.zeros((2, 0, 3, H, W)), torch.zeros((0, 3, H, W))
    return torch.stack(gts), torch.stack(blocks, dim=1), torch.stack(lasts)


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c0, c1 = chain_range(TOTAL, world, rank)
        gt, blocks, last = _run_chains(c0, c1)
        s, n = reduce_psnr(blocks, gt, world)
        full_last = gather_chains(last, TOTAL, world)
        full_gt = gather_chains(gt, TOTAL, world)
        torch.save({"psnr_sum": s, "n": n, "last": full_last, "gt": full_gt}, os.path.join(out_dir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    gt, blocks, last = _run_chains(0, TOTAL)
    ref_psnr = psnr(gt, blocks.mean(dim=0)).sum().item()
    for r in range(world):
        got = torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True)
        assert got["n"] == TOTAL
        assert abs(got["psnr_sum"] - ref_psnr) < 1e-9 * max(1.0, abs(ref_psnr))
        assert torch.equal(got["last"], last)        # bit-identical per chain, any split
        assert torch.equal(got["gt"], gt)


def _fake_record(i):
    """A result record shaped like metrics.analyse_run's + the run parameters (sampling_images.py:409-470)."""
    import numpy as np
    rng = np.random.default_rng(100 + i)
    h, w = (6, 5) if i % 2 else (5, 7)                 # two image shapes, as CBSD68's two orientations
    rec = {"PSNR_sample": [float(v) for v in rng.normal(20, 1, 4)], "SIM_sample": [float(v) for v in rng.random(4)],
           "PSNR_mmse": [float(v) for v in rng.normal(25, 1, 3)], "SIM_list": [],
           "observation": rng.random((h, w, 3), dtype=np.float32), "init": rng.random((h, w, 3), dtype=np.float32),
           "PSNR_y": float(rng.normal(8, 1)), "SIM_y": 0.1 * i, "ground_truth": rng.random((h, w, 3), dtype=np.float32),
           "MMSE": rng.random((h, w, 3), dtype=np.float32), "PSNR_MMSE": 27.0 + i, "SIM_MMSE": 0.8,
           "std": rng.random((h, w, 3)).astype(np.float32), "diff": rng.random((h, w, 3)),   # float64 too
           "n_iter": 1000, "s": 10 / 255.0, "alpha": 1.0, "sigma": 1.0, "l": 4, "lambda": 10.0, "delta": 1.5e-3}
    mask = torch.from_numpy(rng.random((1, 3, h, w)) > 0.5).to(torch.int64)
    return rec, mask, f"sigma1.0_s10_{i}"


N_IMAGES = 5


def _records_worker(rank, world, port, out_dir, backend="gloo"):
    from psgla_for_posterior_sampling_amd.sharding import gather_records, reduce_dataset_psnr
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = "cpu"
    if backend == "nccl":                    # one GPU per rank (RCCL refuses two ranks on one device)
        torch.cuda.set_device(rank)
        dev = f"cuda:{rank}"
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        a, b = chain_range(N_IMAGES, world, rank)
        local = {i: _fake_record(i) for i in range(a, b)}
        s, q, n = reduce_dataset_psnr(local, world, dev)
        got = gather_records(local, world, rank, dev)
        torch.save({"sum": s, "n": n, "none": got is None}, os.path.join(out_dir, f"s{rank}.pt"))
        if rank == 0:
            import pickle
            with open(os.path.join(out_dir, "records.pkl"), "wb") as f:   # written and read by this test only
                pickle.dump(got, f)
    finally:
        dist.destroy_process_group()


def _check_records_gather(tmp_path, backend):
    import pickle
    import numpy as np
    world = 2
    mp.start_processes(_records_worker, args=(world, _free_port(), str(tmp_path), backend), nprocs=world,
                       join=True, start_method="spawn")
    with open(os.path.join(tmp_path, "records.pkl"), "rb") as f:
        got = pickle.load(f)
    assert sorted(got) == list(range(N_IMAGES))
    for i in range(N_IMAGES):
        rec, mask, name = _fake_record(i)
        grec, gmask, gname = got[i]
        assert gname == name and set(grec) == set(rec)
        for k, v in rec.items():
            if isinstance(v, np.ndarray):
                assert grec[k].dtype == v.dtype and np.array_equal(grec[k], v), k
            else:
                assert type(grec[k]) is type(v) and grec[k] == v, k
        assert gmask.dtype == mask.dtype and torch.equal(gmask, mask)
    for r in range(world):
        s = torch.load(os.path.join(tmp_path, f"s{r}.pt"), weights_only=True)
        assert s["n"] == N_IMAGES
        assert abs(s["sum"] - sum(27.0 + i for i in range(N_IMAGES))) < 1e-9
        assert s["none"] == (r != 0)


def test_two_rank_records_gather_exact(tmp_path):
    """The sharded CLI's result path (sampling_images.main, world > 1): per-image records gathered to rank 0
    through one float64 tensor per rank plus gather_object metadata -- every array, list, scalar, dtype and
    the mask come back identical; the dataset PSNR all_reduce counts every image once; other ranks get None."""
    _check_records_gather(tmp_path, "gloo")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="the RCCL path needs two GPUs (one rank per device)")
def test_two_rank_records_gather_exact_nccl(tmp_path):
    """The same gather over RCCL (dist_backend's choice on a multi-GPU node): the float64 transport tensors
    live on each rank's device."""
    _check_records_gather(tmp_path, "nccl")
