#!/usr/bin/env python3
"""Throughput of the DNN-denoiser configurations (BASELINE.json configs[2..4]; not the headline line).

    python tools/bench_dnn.py --workload dncnn-inpaint|dncnn-deblur|drunet-ula [--batch 64] [--steps 20]

Random-init networks (no weights offline), synthetic U[0,1) 3x256x256 images, the reference's
parameters (sampling_images.py:100-198): DnCNN s = 2/255, lambda = 5; PnP-ULA + DRUNet s1 = 5/255.
Steps are hipGraph-replayed (engine.DenoiserChains / UlaChains).  Prints one JSON line: chain-steps/s,
the denoiser's algorithmic TFLOP/s (layer-shape FLOPs, denoisers.py) against the fp32 peak, and the
denoiser forward timed alone with HIP events.  The HIP passes' own durations come from a rocprofv3 kernel trace
of this command (tools/dnn_pass_roofline.py), not from a difference of wall times."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md (vector = matrix f32 peak)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="dncnn-inpaint", choices=["dncnn-inpaint", "dncnn-deblur", "drunet-ula"])
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--H", type=int, default=256)
    p.add_argument("--W", type=int, default=256)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--graph-steps", type=int, default=10)
    p.add_argument("--find", action="store_true", help="torch.backends.cudnn.benchmark (MIOpen find)")
    p.add_argument("--channels-last", action="store_true")
    a = p.parse_args()
    torch.backends.cudnn.benchmark = a.find
    from psgla_for_posterior_sampling_amd import hip_ops as K
    from psgla_for_posterior_sampling_amd.denoisers import (DenoiserPrior, DnCNN, DRUNet, dncnn_flops_per_pixel,
                                                            drunet_flops_per_pixel)
    from psgla_for_posterior_sampling_amd.engine import DenoiserChains, UlaChains
    from psgla_for_posterior_sampling_amd.fidelity import deblurring_problem, inpainting_problem
    dev = torch.device("cuda:0")
    B, C, H, W = a.batch, 3, a.H, a.W
    g = torch.Generator(device=dev).manual_seed(1234)
    xs = torch.rand((B, C, H, W), generator=g, device=dev)
    torch.manual_seed(0)
    n_iter = 4 + a.steps + 2 * a.graph_steps
    if a.workload.startswith("dncnn"):
        den = DnCNN(device=dev)
        flops = dncnn_flops_per_pixel() * H * W
        s, lam = 2 / 255.0, 5.0
        delta = 6.1515e-5
        if a.workload == "dncnn-inpaint":
            dg, y, init, _, _ = inpainting_problem(xs, seed_ip=0)
        else:
            dg, y, init = deblurring_problem(xs, seed_ip=0, l=4)
        c1 = float((torch.tensor(delta).float() / torch.tensor(lam).float()).item())
        c2 = float((torch.tensor(np.sqrt(2)).float() * torch.tensor(s).float()).item())
        eng = DenoiserChains(init.contiguous(), dg, den, torch.tensor(s, device=dev), alpha=1.0, c1=c1, c2=c2, seed=0,
                             n_iter=n_iter, n_inter=10, n_inter_mmse=10)
    else:
        den = DRUNet(device=dev)
        flops = drunet_flops_per_pixel() * H * W
        s1 = 5 / 255.0
        dg, y, init, _, _ = inpainting_problem(xs, seed_ip=0)
        prior = DenoiserPrior(den, s1, torch.tensor(1.0, device=dev), torch.tensor(s1 ** 2, device=dev))
        delta, lam = 1.00122e-6, 3.7693e-6
        brw = float(torch.sqrt(torch.tensor(2 * delta, dtype=torch.float32).double()).float())
        eng = UlaChains(init.contiguous(), dg, prior, delta=delta, lambd=lam, brw=brw, c_min=-1.0, c_max=2.0, seed=0,
                        n_iter=n_iter, n_inter=1000, n_inter_mmse=1000)
    if a.channels_last:
        den.to(memory_format=torch.channels_last)
    eng.step(2)
    eng.capture(a.graph_steps)
    eng.replay(1)
    torch.cuda.synchronize()
    reps = max(1, a.steps // eng.graph_steps)
    t0 = time.perf_counter()
    eng.replay(reps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = reps * eng.graph_steps
    ms = dt / steps * 1e3
    # the denoiser forward alone (eager), to split the step
    x = torch.rand((B, C, H, W), device=dev)
    if a.channels_last:
        x = x.to(memory_format=torch.channels_last)
    with torch.no_grad():
        den.forward(x, 0.01)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            den.forward(x, 0.01)
        e1.record()
        e1.synchronize()
    den_ms = e0.elapsed_time(e1) / 3
    tflops = flops * B / (den_ms * 1e-3) / 1e12
    print(json.dumps({
        "workload": a.workload, "chains": B, "image": [C, H, W], "steps": steps,
        "ms_per_step": round(ms, 3), "chain_steps_per_s": round(B * steps / dt, 2),
        "denoiser_ms": round(den_ms, 3), "denoiser_gflop_per_image": round(flops / 1e9, 2),
        "denoiser_tflops": round(tflops, 1), "fp32_peak_tflops": FP32_PEAK_TFLOPS,
        "denoiser_frac_of_peak": round(tflops / FP32_PEAK_TFLOPS, 3),
        "miopen_find": a.find, "channels_last_flag": a.channels_last, "dtype": "f32", "weights": "random-init (none offline)",
    }), flush=True)


if __name__ == "__main__":
    main()
