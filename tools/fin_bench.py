"""Time the per-step finaliser kernel alone (launch_mask = 2), HIP events on its stream."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psgla_for_posterior_sampling_amd import _native as N  # noqa: E402
from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402
from psgla_for_posterior_sampling_amd.engine import FusedTvChains  # noqa: E402

dev = torch.device("cuda:0")
B, C, H, W = 64, 3, 256, 256
x = torch.rand((B, C, H, W), device=dev)
m = (torch.rand((H, W), device=dev) > 0.5).to(torch.uint8)
eng = FusedTvChains(x, x, m, c1=1e-4, c2=0.05, sigma2=1.5e-5, alpha=1.0, ths=0.04, tv=K.TvConstants(n_it_max=10),
                    seed=0, n_iter=20, n_inter=10, n_inter_mmse=10)
eng.step(2)
d = N.PsglaTvStep.from_buffer_copy(eng.desc)
d.launch_mask = 2
d.advance_step = 0
for _ in range(5):
    eng._launch(d)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200):
    eng._launch(d)
e1.record()
e1.synchronize()
print("finaliser us per launch: %.2f" % (e0.elapsed_time(e1) / 200 * 1e3))
