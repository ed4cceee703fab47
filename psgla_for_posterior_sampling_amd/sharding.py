"""Chain sharding over GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The reference runs one chain per image, sequentially (sampling_images.py:265); chains never
interact.  Here a batch of chains is split contiguously over ranks; every chain keeps its
GLOBAL id, which keys its noise stream, so a chain's trajectory is bitwise independent of the
number of GPUs (tests/test_gpu_parity.py::test_fused_chains_independent_of_batching_and_graph,
tests/test_sharding_gloo.py).  The only collectives are the final ones: all_reduce of per-chain
PSNR sums and all_gather of per-chain MMSE images -- no per-step communication.
"""
from __future__ import annotations

import math

import torch


def chain_range(total: int, world: int, rank: int):
    """Contiguous [start, end) chain ids of `rank` (sizes differ by at most one)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    base, rem = divmod(int(total), int(world))
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def mmse_of_blocks(blocks: torch.Tensor) -> torch.Tensor:
    """MMSE = mean of the block means (sampling_images.py:412, :428), per chain.  blocks: (nb, B, ...)."""
    return blocks.mean(dim=0)


def psnr(gt: torch.Tensor, x: torch.Tensor, data_range: float = 1.0) -> torch.Tensor:
    """Per-chain PSNR in dB (skimage.metrics.peak_signal_noise_ratio, data_range=1), fp64."""
    dims = tuple(range(1, gt.dim()))
    mse = ((gt.double() - x.double()) ** 2).mean(dim=dims)
    return 10.0 * torch.log10((data_range ** 2) / mse)


def reduce_psnr(blocks: torch.Tensor | None, gt: torch.Tensor, world: int):
    """Sum over ALL chains of the MMSE PSNR, and the chain count (RCCL all_reduce when world > 1)."""
    if blocks is None or blocks.shape[0] == 0:
        vals = torch.zeros(2, dtype=torch.float64, device=gt.device)
    else:
        p = psnr(gt, mmse_of_blocks(blocks))
        vals = torch.stack([p.sum(), torch.tensor(float(p.numel()), dtype=torch.float64, device=gt.device)])
    if world > 1:
        import torch.distributed as dist
        if dist.get_backend() == "gloo":        # gloo: host tensors (CPU tests, single-GPU rehearsals)
            vals = vals.cpu()
        dist.all_reduce(vals, op=dist.ReduceOp.SUM)
    s, n = vals.tolist()
    return s, int(round(n)) if not math.isnan(n) else 0


def gather_chains(local: torch.Tensor, total: int, world: int):
    """all_gather of per-chain tensors (B_local, ...) into (total, ...) on every rank."""
    if world == 1:
        return local
    import torch.distributed as dist
    per = -(-total // world)
    dev = "cpu" if dist.get_backend() == "gloo" else local.device
    buf = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    buf[: local.shape[0]] = local
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf)
    parts = []
    for r in range(world):
        a, b = chain_range(total, world, r)
        parts.append(out[r][: b - a])
    return torch.cat(parts, dim=0).to(local.device)
