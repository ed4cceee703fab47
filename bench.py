#!/usr/bin/env python3
"""Langevin-step throughput of the fused PSGLA+TV HIP step (BASELINE.json configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 64] [--scaling strong|weak]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Workload (config.workload): PSGLA, inpainting 50 %, TV denoiser (deepinv TVDenoiser,
n_it_max=10, warm-started), s = 10/255, lambda = 10, delta = s^2, sigma = 1/255,
n_inter = n_inter_mmse = 10 (the N = 10000 TV settings of sampling_images.py:180-198),
synthetic 3x256x256 fp32 images (one per chain, U[0,1) from the device generator seeded
1234 + chain id), the reference's shared inpainting mask (torch.rand on the device
generator, seed_ip = 0, > 0.5).

Scaling: strong by default -- a batch of 64 chains in total, split
contiguously over the N ranks (64/N chains per GPU); `--scaling weak` keeps 64 chains per GPU.
Chains are independent: no collective in the step; chain ids are global, so every chain's
samples are the same for any N.  One RCCL all_reduce after the timed region combines the
per-chain MMSE PSNR.

Timed region: exactly K steps (K // G hipGraph replays of G-step graphs + K % G eager launches;
the device step counter advances the noise counter, block-mean coefficients and sample /
block slots), barrier + synchronize on both sides, max over ranks.  value = chain-steps
(image-steps of 3x256x256) per second over all GPUs.

Warm-up: the W steps (eager + graph capture), then untimed graph replays until at least
--warmup-seconds of GPU work have run (clocks and power state settle; reported as
`warmup_s`), after which the chain state, accumulators, TV state and step index are restored
from a snapshot taken before them: the timed steps are exactly those of a run that warmed up
for W steps, on every rank, whatever the wall-clock warm-up ran.

The roofline figure divides the algorithmic bytes of one launch by the dominant kernel's
(tv_stream_kernel at 64 chains per GPU, tv_tile_kernel at 8: one launch per step) average duration from HIP events recorded on the
replay stream around the timed region (the committed rocprofv3 kernel trace of the same command agrees
with it).  `traffic` (HBM bytes per launch
from rocprofv3 PMC counters) cannot be collected inside an un-profiled run: it is read from
the committed profile named in `traffic_source`, measured at the commit it records.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Langevin steps/sec (3×256×256, batch=64) at 1/2/4/8 GPU; HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# committed PMC summaries (tools/profile_round.sh + tools/pmc_summary.py) by dominant kernel
PMC_PROFILES = {"tv_stream_kernel": os.path.join("profiles", "r06zi_pmc_tv_stream.json"),
                "tv_tile_kernel": os.path.join("profiles", "r06zi_pmc_tv_tile.json")}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=400)
    p.add_argument("--warmup", type=int, default=40)
    p.add_argument("--warmup-seconds", type=float, default=1.5,
                   help="minimum untimed GPU work (graph replays) before the timed steps")
    p.add_argument("--batch", type=int, default=64, help="chains in total (strong) or per GPU (weak)")
    p.add_argument("--scaling", choices=["weak", "strong"], default="strong")
    p.add_argument("--H", type=int, default=256)
    p.add_argument("--W", type=int, default=256)
    p.add_argument("--graph-steps", type=int, default=20)
    p.add_argument("--exact", action="store_true", help="bit-exact (IEEE div/sqrt) TV kernel")
    p.add_argument("--tv-iters", type=int, default=10, help="TV n_it_max (analysis only; the workload is 10)")
    p.add_argument("--tv-tol", type=float, default=1e-5, help="TV early-stop tolerance (analysis only; the workload "
                   "is deepinv's 1e-5, where the stop never fires; a large value makes it fire every step)")
    p.add_argument("--serial-redo", action="store_true", help="early-stop recompute by the finalising workgroup "
                   "alone (the pre-ABI-11 path; analysis only)")
    p.add_argument("--stream-wgs", type=int, default=0, help="stream kernel work split (0 auto, -1 per plane)")
    p.add_argument("--stream-windows", choices=["auto", "whole", "half"], default="auto",
                   help="stream kernel column windows (auto: half-wave windows where they idle fewer lanes; "
                        "half: always, a diagnostic)")
    p.add_argument("--variant", choices=["auto", "band", "stream", "tile"], default="auto",
                   help="fused TV kernel (analysis; auto = the library's choice)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the batch-1 CPU leg")
    p.add_argument("--cpu-b64-steps", type=int, default=10, help="timed steps of the batch-64 CPU leg (0: skip)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--pmc-json", default=None, help="PMC summary to report as roofline.traffic (default: the "
                   "committed profile of the dispatched kernel, when it was measured on this workload)")
    return p.parse_args()


def algorithmic_bytes_per_launch(B, C, H, W, step0, steps, n_inter, nm):
    """Compulsory HBM bytes of one fused-step kernel launch, averaged over the timed steps.
    Per element: read X 4 + u2 8 + y 4 (+ mean 4 + sq 4 unless the block restarts), write
    X 4 + u2 8 + mean 4 + sq 4 (block means instead of the live accumulators at a block
    end), + the sample copy 4 every n_inter steps; + the (H,W) u8 mask once per launch."""
    E = B * C * H * W
    tot = 0.0
    per = nm + 1
    for i in range(step0, step0 + steps):
        b = 4 + 8 + 4 + 4 + 8 + 8       # X r/w, u2 r/w, y r, mean+sq w (or block w)
        if i % per != 0:
            b += 8                       # mean + sq read
        if i % n_inter == 0:
            b += 4                       # sample store
        tot += b * E + H * W
    return tot / steps


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds: float, b64_steps: int):
    """The reference algorithm on the host cores: oracle/ (op-for-op torch-CPU restatement of
    restoration_algorithms.py:231-271 + the deepinv TV prox, pinned to the reference by
    tests/golden), at batch 1 (as the reference runs, bounded by `seconds`) and at batch 64
    (the benched workload; `b64_steps` steps, one psgla call -- the reference needs n_iter >= 10)."""
    from oracle import psgla_oracle as orc
    # threads: torch's intra-op pool, i.e. OMP_NUM_THREADS where the harness sets it (the GPU box gives one
    # GPU's job a 16-CPU share of the host; os.cpu_count() there counts the whole machine).  Reported
    # beside the affinity-allowed and logical CPU counts and the cgroup CPU quota.
    threads = torch.get_num_threads()
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    s = 10 / 255.0
    alpha = torch.tensor(1.0)
    lam = torch.tensor(10.0)

    def problem(B):
        g = torch.Generator().manual_seed(1234)
        x = torch.rand((B, 3, 256, 256), generator=g)
        dg, y, init, _ = orc.inpainting_problem(x, seed_ip=0)
        return dg, init

    def run(B, n_iter, tv, X, dg):
        Xl, _, _ = orc.psgla(X, dg, tv, alpha, lam, sig_float=s, delta=s ** 2, n_iter=n_iter, n_inter=10,
                             n_inter_mmse=10, seed=0)
        return Xl[-1][None] if B == 1 else Xl[-1]

    # batch 1: blocks of 10 steps until `seconds` have elapsed (the first block is warm-up)
    dg, X = problem(1)
    tv = orc.TVDenoiser(n_it_max=10)
    X = run(1, 10, tv, X, dg)
    steps, t0 = 0, time.perf_counter()
    while True:
        X = run(1, 10, tv, X, dg)
        steps += 10
        if time.perf_counter() - t0 > seconds:
            break
    dt1 = time.perf_counter() - t0
    b1 = steps / dt1
    out = {"value": round(b1, 2), "unit": "image-steps/s", "cores": threads, "kind": "port",
           "sample": f"batch 1: {steps} PSGLA+TV steps (3x256x256) after 10 warm-up steps, {dt1:.1f} s",
           "batch1_image_steps_per_s": round(b1, 2), "cpu_model": cpu_model(), "threads": threads,
           "host_logical_cpus": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
           "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    if b64_steps > 0:
        dg, X = problem(64)
        tv = orc.TVDenoiser(n_it_max=10)
        n = max(10, int(b64_steps))
        t0 = time.perf_counter()
        run(64, n, tv, X, dg)
        dt = time.perf_counter() - t0
        b64 = 64 * n / dt
        out["batch64_image_steps_per_s"] = round(b64, 2)
        out["batch64_ms_per_step"] = round(dt / n * 1e3, 1)
        out["value"] = round(b64, 2)      # the benched workload's batch
        out["sample"] = (f"batch 64: {n} PSGLA+TV steps (64x3x256x256, one psgla call, after the batch-1 leg) "
                         f"in {dt:.1f} s; " + out["sample"])
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU over RCCL ("nccl"); PSGLA_DIST_BACKEND=gloo rehearses the multi-rank path on a
    # box with fewer GPUs than ranks (ranks then share devices: plumbing only, the timings mean nothing)
    backend = os.environ.get("PSGLA_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local_dev = local % max(ndev, 1)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_dev}"))
        else:
            dist.init_process_group(backend)
    dev = torch.device(f"cuda:{local_dev}")
    torch.cuda.set_device(dev)

    from psgla_for_posterior_sampling_amd import hip_ops as K
    from psgla_for_posterior_sampling_amd.engine import FusedTvChains
    from psgla_for_posterior_sampling_amd.sharding import chain_range

    C, H, W = 3, args.H, args.W
    total_chains = args.batch * world if args.scaling == "weak" else args.batch
    if total_chains < world:
        raise SystemExit(f"{total_chains} chains cannot be split over {world} GPUs")
    c0, c1 = chain_range(total_chains, world, rank)
    B = c1 - c0
    # synthetic per-chain ground truths, the reference's shared mask, observations
    xs = torch.empty((B, C, H, W), device=dev)
    for b in range(B):
        g = torch.Generator(device=dev).manual_seed(1234 + c0 + b)
        xs[b] = torch.rand((C, H, W), generator=g, device=dev)
    gen = torch.Generator(device=dev).manual_seed(0)
    m = torch.rand((H, W), generator=gen, device=dev)
    mask_2d = 1 * (m > 0.5)
    mask = torch.ones(C, device=dev)[None, :, None, None] * mask_2d[None, None]
    sigma1 = 1 / 255.0
    y = mask * xs + torch.normal(torch.zeros_like(xs), std=sigma1 * torch.ones_like(xs), generator=gen)
    init = mask * y + (1 - mask) * 0.5
    s = 10 / 255.0
    lam = 10.0
    delta = s ** 2
    c1f = float((torch.tensor(delta).float() / torch.tensor(lam).float()).item())
    c2f = float((torch.tensor(np.sqrt(2)).float() * torch.tensor(s).float()).item())
    n_inter = nm = 10
    # graphs of an even step count: rewinding the step index after the warm-up keeps the parity
    gs = max(2, min(args.graph_steps, max(args.steps, 2)))
    gs += gs & 1
    w_eager = max(1, args.warmup - gs)
    # steps the schedule is sized for: eager warm-up + one replay, the timed steps
    n_iter = w_eager + gs + args.steps + 8
    eng = FusedTvChains(init.contiguous(), y.contiguous(), mask_2d.to(torch.uint8), c1=c1f, c2=c2f,
                        sigma2=float(np.float32(sigma1 ** 2)), alpha=1.0, ths=float(np.float32(s)),
                        tv=K.TvConstants(n_it_max=args.tv_iters, tol=args.tv_tol), seed=0,
                        n_iter=n_iter, parallel_redo=not args.serial_redo,
                        n_inter=n_inter, n_inter_mmse=nm, chain0=c0, exact=args.exact,
                        stream_wgs=args.stream_wgs, kernel_variant=args.variant, stream_windows=args.stream_windows)
    # warm-up: eager steps + graph capture + one replay
    eng.step(w_eager)
    eng.capture(gs)
    eng.replay(1)
    torch.cuda.synchronize()
    step0 = eng.steps_done
    # time-based warm-up: replays until >= warmup_seconds of GPU work, then the chain state, accumulators
    # and step index are restored to where they were, so the timed steps (and the reported PSNR) are
    # those of a run that warmed up for exactly W steps, whatever the wall-clock warm-up ran
    snap = eng.snapshot()
    tw0 = time.perf_counter()
    n_warm = 0
    while time.perf_counter() - tw0 < args.warmup_seconds:
        for _ in range(5):
            eng.replay(1)
            eng.rewind(step0, discard_pending=True)        # (restored from the snapshot below)
            n_warm += gs
        torch.cuda.synchronize()
    warmup_s = time.perf_counter() - tw0
    eng.restore(snap)
    del snap
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    steps = args.steps
    reps, rem = divmod(steps, gs)
    barrier()
    torch.cuda.synchronize()
    # HIP events on the stream the graphs (one tv_stream_kernel launch per step) are replayed on
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    eng.replay(reps)
    eng.step(rem)
    eng.settle()                                     # the last step's early-stop redo, if one is pending
    ev1.record()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    live_kern_ms = ev0.elapsed_time(ev1) / steps     # kernel + its launch boundary, in the timed region
    eng.check_handoff()                              # the tile kernel's early-stop guard (after the timed region)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    alg_bytes = algorithmic_bytes_per_launch(B, C, H, W, step0, steps, n_inter, nm)
    achieved = alg_bytes / (live_kern_ms * 1e-3) / 1e9

    # ---- final reduction (RCCL): per-chain MMSE PSNR of the blocks so far ----
    from psgla_for_posterior_sampling_amd.sharding import reduce_psnr
    blocks, _ = eng.blocks()
    psnr_sum, n_chains = reduce_psnr(blocks, xs, world)

    # ---- placement: every rank's device and PCI address, gathered to rank 0 (small metadata) ----
    props = torch.cuda.get_device_properties(dev)
    here = {"rank": rank, "local_rank": local, "device": torch.cuda.current_device(),
            "pci": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}",
            "chains": [c0, c1]}
    placement = [here]
    if world > 1:
        import torch.distributed as dist
        placement = [None] * world
        dist.all_gather_object(placement, here)

    traffic, traffic_info = None, None
    kname = eng.main_kernel            # the kernel the timed graphs launch, once per step
    pmc_json = args.pmc_json or os.path.join(REPO, PMC_PROFILES.get(kname, "none"))
    if os.path.exists(pmc_json):
        try:
            pj = json.load(open(pmc_json))
            if (pj.get("kernel") == kname and pj.get("workload", {}).get("chains_per_gpu") in (None, B)
                    and pj.get("exact", False) == args.exact
                    and args.tv_iters == 10 and args.tv_tol == 1e-5 and (H, W) == (256, 256)):
                traffic = pj.get("hbm_bytes_per_launch")
                traffic_info = {"traffic_source": os.path.relpath(pmc_json, REPO),
                                "traffic_commit": pj.get("commit"),
                                "traffic_note": "rocprofv3 PMC (FETCH_SIZE x2 + WRITE_SIZE), not measured in this run"}
        except Exception:
            traffic = None

    if rank == 0:
        # the CPU baseline is timed at N = 1 only (rank 0 alone on the host); multi-GPU lines carry null
        cpu = None if (args.no_cpu or world > 1) else cpu_baseline(args.cpu_seconds, args.cpu_b64_steps)
        value = total_chains * steps / dt
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": kname, "kernel_ms": round(live_kern_ms, 5), "algorithmic_bytes_per_launch": int(alg_bytes)}
        if traffic_info:
            roof.update(traffic_info)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "image-steps/s (chain-steps of 3x256x256, summed over GPUs)",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "warmup_s": round(warmup_s, 3),
            "warmup_replayed_steps": n_warm,
            "ms_per_step": round(dt / steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (U[0,1) images per chain, reference mask/observation recipe)",
            "config": {"workload": "psgla+TV inpainting 50% (BASELINE configs[1]), n_it_max=10",
                       "dist_backend": backend if world > 1 else None,
                       "global_batch": total_chains, "chains_per_gpu": B, "image": [C, H, W],
                       "parallelism": f"chains{world}", "graph_steps": gs,
                       "kernel_mode": "exact" if args.exact else "fast",
                       "tv_tol": args.tv_tol, "early_stop_redo": "serial" if args.serial_redo else "parallel",
                       "batch_steps_per_s": round(steps / dt, 2)},
            "roofline": roof,
            "cpu_baseline": cpu,
            "mmse_psnr_mean_db": round(psnr_sum / max(n_chains, 1), 3),
        }
        if world > 1:
            line["config"]["placement"] = placement
            line["config"]["distinct_gpus"] = len({p["pci"] for p in placement})
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
