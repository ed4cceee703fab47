"""Profiling driver: the bench workload (64 chains x 3x256x256 PSGLA+TV), N eager steps.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 tools/prof_step.py
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402
from psgla_for_posterior_sampling_amd.engine import FusedTvChains  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--steps", type=int, default=30)
p.add_argument("--batch", type=int, default=64)
p.add_argument("--exact", action="store_true")
p.add_argument("--main-only", type=int, default=0, help="extra tile-kernel-only launches")
p.add_argument("--stream-wgs", type=int, default=0)
p.add_argument("--tv-iters", type=int, default=10)
a = p.parse_args()
dev = torch.device("cuda:0")
B, C, H, W = a.batch, 3, 256, 256
g = torch.Generator(device=dev).manual_seed(1234)
xs = torch.rand((B, C, H, W), generator=g, device=dev)
gen = torch.Generator(device=dev).manual_seed(0)
mask_2d = 1 * (torch.rand((H, W), generator=gen, device=dev) > 0.5)
mask = mask_2d[None, None].float()
y = mask * xs + torch.normal(torch.zeros_like(xs), std=(1 / 255.0) * torch.ones_like(xs), generator=gen)
init = mask * y + (1 - mask) * 0.5
s = 10 / 255.0
c1 = float((torch.tensor(s * s).float() / torch.tensor(10.0)).item())
c2 = float((torch.tensor(np.sqrt(2)).float() * torch.tensor(s).float()).item())
eng = FusedTvChains(init.contiguous(), y.contiguous(), mask_2d.to(torch.uint8), c1=c1, c2=c2,
                    sigma2=float(np.float32((1 / 255.0) ** 2)), alpha=1.0, ths=float(np.float32(s)),
                    tv=K.TvConstants(n_it_max=a.tv_iters), seed=0, n_iter=a.steps, n_inter=10, n_inter_mmse=10,
                    exact=a.exact, stream_wgs=a.stream_wgs)
eng.step(a.steps)
if a.main_only:
    eng.launch_main_only(a.main_only)
torch.cuda.synchronize()
print("done", eng.steps_done, float(eng.X.mean()))
