"""Chain sharding over GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The reference runs one chain per image, sequentially (sampling_images.py:265); chains never
interact.  Here a batch of chains is split contiguously over ranks; every chain keeps its
GLOBAL id, which keys its noise stream, so a chain's trajectory is bitwise independent of the
number of GPUs (tests/test_gpu_parity.py::test_fused_chains_independent_of_batching_and_graph,
tests/test_sharding_gloo.py).  The only collectives are the final ones: all_reduce of per-chain
PSNR sums and all_gather of per-chain MMSE images (bench), and for the sharded CLI the gather of the
per-image result arrays to rank 0 plus the dataset PSNR all_reduce (RCCL on device tensors when every
rank has its own GPU) -- no per-step communication.
"""
from __future__ import annotations

import math
import os

import numpy as np
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


def dist_backend(local_world: int) -> str:
    """Backend of the sharded CLI's process group: "nccl" (RCCL over xGMI) when every rank of this node has a
    GPU of its own, else "gloo" (the one-GPU rehearsal: RCCL cannot put two ranks on one device).
    PSGLA_DIST_BACKEND overrides.  torch.cuda.device_count() does not initialise the GPU."""
    env = os.environ.get("PSGLA_DIST_BACKEND")
    if env:
        return env
    return "nccl" if torch.cuda.device_count() >= max(int(local_world), 1) else "gloo"


def _split_record(rec: dict):
    """(arrays, meta): every float array (and list of floats) of a result record to go through the tensor
    collective, everything else (scalars, strings) as metadata."""
    arrays, meta = {}, {}
    for k, v in rec.items():
        if isinstance(v, np.ndarray) and v.dtype.kind == "f":
            arrays[k] = ("nd", v)
        elif isinstance(v, torch.Tensor):
            arrays[k] = ("torch", v.detach().cpu().numpy())
        elif isinstance(v, list) and v and all(isinstance(x, float) for x in v):
            arrays[k] = ("list", np.asarray(v, dtype=np.float64))
        else:
            meta[k] = v
    return arrays, meta


def gather_records(local: dict, world: int, rank: int, device, obj_group=None):
    """Gather the sharded CLI's per-image results to rank 0 (sampling_images.py:409-470 per image; only rank 0
    writes them).  `local` maps image index -> (record dict, mask tensor or None, name).  The arrays (MMSE, std,
    observation, the PSNR / SSIM curves, the mask ...) travel as ONE float64 tensor per rank through a
    tensor gather on the process group's backend -- device tensors over RCCL when it is "nccl" -- and only the
    small metadata (keys, shapes, dtypes, scalars) through gather_object on `obj_group` (gloo).  float32 values
    survive the float64 transport exactly.  Returns the merged dict on rank 0, None on the other ranks."""
    import torch.distributed as dist
    if world == 1:
        return dict(local)
    nccl = dist.get_backend() == "nccl"
    dev = torch.device(device) if nccl else torch.device("cpu")
    chunks, meta = [], []
    off = 0
    for i in sorted(local):
        rec, mask, name = local[i]
        arrays, m = _split_record(rec)
        if mask is not None:
            arrays["__mask__"] = ("torch", mask.detach().cpu().numpy())
        layout = {}
        for k, (kind, a) in arrays.items():
            if a.dtype.kind in "iub" and a.size and int(np.abs(a.astype(np.int64)).max()) >= 2 ** 53:
                raise ValueError(f"gather_records: integer array {k!r} has values beyond 2**53 (float64 transport)")
            flat = np.ascontiguousarray(a, dtype=np.float64).reshape(-1)
            layout[k] = (kind, str(a.dtype), tuple(a.shape), off, flat.size)
            chunks.append(flat)
            off += flat.size
        meta.append((i, name, m, layout))
    payload = torch.from_numpy(np.concatenate(chunks) if chunks else np.zeros(0)).to(dev)
    n = torch.tensor([payload.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    nmax = max(int(s.item()) for s in sizes)
    buf = torch.zeros(nmax, dtype=torch.float64, device=dev)
    buf[: payload.numel()] = payload
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, parts, dst=0)
    metas = [None] * world if rank == 0 else None
    dist.gather_object(meta, metas, dst=0, group=obj_group)
    if rank != 0:
        return None
    out = {}
    for r in range(world):
        host = parts[r][: int(sizes[r].item())].cpu().numpy()
        for i, name, m, layout in metas[r]:
            rec = dict(m)
            mask = None
            for k, (kind, dtype, shape, o, cnt) in layout.items():
                a = host[o:o + cnt].astype(dtype).reshape(shape)
                if k == "__mask__":
                    mask = torch.from_numpy(a)
                elif kind == "list":
                    rec[k] = [float(x) for x in a]
                elif kind == "torch":
                    rec[k] = torch.from_numpy(a)
                else:
                    rec[k] = a
            out[i] = (rec, mask, name)
    return out


def reduce_dataset_psnr(records: dict, world: int, device):
    """The dataset summary over all ranks' images: (sum of PSNR_MMSE, sum of SIM_MMSE, image count), one
    all_reduce(SUM) of a 3-element float64 tensor (on the device over RCCL when the backend is nccl)."""
    vals = torch.tensor([sum(r[0]["PSNR_MMSE"] for r in records.values()),
                         sum(r[0]["SIM_MMSE"] for r in records.values()), float(len(records))], dtype=torch.float64)
    if world > 1:
        import torch.distributed as dist
        vals = vals.to(torch.device(device) if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(vals, op=dist.ReduceOp.SUM)
    s, q, n = vals.tolist()
    return s, q, int(round(n))


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
