"""Per-kernel timing of the generic (opaque-closure) HIP kernels at the BASELINE size
(64 chains x 3x256x256 fp32), HIP events on the launching stream.  One JSON line per kernel:
time per launch, algorithmic HBM bytes per launch and the resulting GB/s (8 TB/s roofline).

    python3 tools/bench_kernels.py [--batch 64] [--iters 50]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=64)
p.add_argument("--iters", type=int, default=50)
p.add_argument("--l", type=int, default=4)
a = p.parse_args()
dev = torch.device("cuda:0")
B, C, H, W = a.batch, 3, 256, 256
E = B * C * H * W
g = torch.Generator(device=dev).manual_seed(0)
X = torch.rand((B, C, H, W), generator=g, device=dev)
y = torch.rand((B, C, H, W), generator=g, device=dev)
D = torch.rand((B, C, H, W), generator=g, device=dev)
gr = torch.rand((B, C, H, W), generator=g, device=dev)
out = torch.empty_like(X)
mean, sq = torch.zeros_like(X), torch.zeros_like(X)
mask = (torch.rand((H, W), generator=g, device=dev) > 0.5).to(torch.uint8)
h = np.full((2 * a.l + 1, 2 * a.l + 1), 1.0 / (2 * a.l + 1) ** 2)
hc = h.astype(np.float32)
sched = K.Schedule((B, C, H, W), 10 ** 6, 10, 10, dev, store_samples=False, store_blocks=False)


def timed(fn, nbytes, name, flops=None):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.iters):
        fn()
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    line = {"kernel": name, "ms": round(ms, 5), "bytes_per_launch": int(nbytes),
            "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1), "frac_of_8TBps": round(nbytes / (ms * 1e-3) / 8e12, 4)}
    if flops:
        line["TFLOPs"] = round(flops / (ms * 1e-3) / 1e12, 2)
    print(json.dumps(line), flush=True)


s2 = float(np.float32((1 / 255.0) ** 2))
taps = (2 * a.l + 1) ** 2
timed(lambda: K.blur_langevin(X, y, hc, hc, a.l, s2, 1e-4, 0.05, 0, 0, 5, out=out), 12 * E,
      f"blur_grad+langevin (l={a.l})", flops=2 * 2 * taps * E)
timed(lambda: K.blur_grad(X, y, hc, hc, a.l, s2, out=out), 12 * E, f"blur_grad (l={a.l})", flops=2 * 2 * taps * E)
timed(lambda: K.langevin_update(X, gr, 1e-4, 0.05, 0, 0, 5, out=out), 12 * E, "langevin_update")
timed(lambda: K.inpaint_grad(X, y, mask, s2, out=out), 12 * E + H * W, "inpaint_grad")
timed(lambda: K.relax_accumulate(X, D, out, 1.0, mean, sq, sched, 3), 28 * E, "relax_accumulate (alpha=1)")
timed(lambda: K.pnpula_update(X, D, gr, out, 1e-6, 4e-6, 1.4e-3, -1.0, 2.0, mean, sq, sched, 3, 0, 0), 32 * E,
      "pnpula_update")
