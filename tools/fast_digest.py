"""Digest of a short fast-mode PSGLA+TV run (samples, block means, TV state) for comparing two
builds bit for bit: PSGLA_LIB=exp_libs/lib_X.so python tools/fast_digest.py"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402
from psgla_for_posterior_sampling_amd.engine import FusedTvChains  # noqa: E402

dev = torch.device("cuda:0")
B, C, H, W = 8, 3, 256, 256
g = torch.Generator(device=dev).manual_seed(5)
x = torch.rand((B, C, H, W), generator=g, device=dev)
m = (torch.rand((H, W), generator=g, device=dev) > 0.5)
y = m * x + torch.normal(torch.zeros_like(x), std=1 / 255.0, generator=g)
init = m * y + (~m) * 0.5
s = 10 / 255.0
h = hashlib.sha256()
for wgs, variant, exact in ((0, "auto", False), (-1, "stream", False), (0, "stream", False), (0, "tile", True),
                           (0, "stream", True)):
    eng = FusedTvChains(init.contiguous(), y.contiguous(), m.to(torch.uint8), c1=float(s * s / 10.0),
                        c2=float(2 ** 0.5 * s), sigma2=(1 / 255.0) ** 2, alpha=1.0, ths=s,
                        tv=K.TvConstants(n_it_max=10), seed=1, n_iter=40, n_inter=10, n_inter_mmse=10,
                        exact=exact, stream_wgs=wgs, kernel_variant=variant)
    eng.run(40, graph_steps=0)
    torch.cuda.synchronize()
    bm, bm2 = eng.blocks()
    for t in (eng.samples(), bm, bm2, eng.u2_state):
        h.update(t.detach().cpu().numpy().tobytes())
print(os.environ.get("PSGLA_LIB", "default"), h.hexdigest())
