"""Diagnostic: per-role work / wait cycles of the streaming TV kernel (stamps build).

    PSGLA_HIPCC_EXTRA=-DPSGLA_STAMPS -> psgla_for_posterior_sampling_amd/libpsgla_hip_stamps.so
    python3 tools/stamps.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PSGLA_LIB", os.path.join(REPO, "psgla_for_posterior_sampling_amd", "libpsgla_hip_stamps.so"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402
from psgla_for_posterior_sampling_amd.engine import FusedTvChains  # noqa: E402

dev = torch.device("cuda:0")
B, C, H, W = int(os.environ.get("B", "64")), 3, 256, 256
g = torch.Generator(device=dev).manual_seed(1234)
xs = torch.rand((B, C, H, W), generator=g, device=dev)
gen = torch.Generator(device=dev).manual_seed(0)
mask_2d = 1 * (torch.rand((H, W), generator=gen, device=dev) > 0.5)
y = mask_2d * xs
init = mask_2d * y + (1 - mask_2d) * 0.5
s = 10 / 255.0
eng = FusedTvChains(init.contiguous().float(), y.contiguous().float(), mask_2d.to(torch.uint8), c1=1.5379e-4 * 10 / 10,
                    c2=0.0554594, sigma2=float(np.float32((1 / 255.0) ** 2)), alpha=1.0, ths=float(np.float32(s)),
                    tv=K.TvConstants(n_it_max=10), seed=0, n_iter=10, n_inter=10, n_inter_mmse=10)
stamps = torch.zeros((B * C * 32,), dtype=torch.int64, device=dev)
eng.desc.debug_stamps = stamps.data_ptr()
eng.step(5)
torch.cuda.synchronize()
st = stamps.cpu().numpy().astype(np.float64).reshape(B * C, 16, 2)
nsteps = H + 4 + 30
roles = {"front": range(0, 4), "stage": range(4, 14), "back": range(14, 16)}
for name, ws in roles.items():
    wk = st[:, list(ws), 0].mean() / nsteps
    wt = st[:, list(ws), 1].mean() / nsteps
    print(f"{name:6s} work/step {wk:8.1f} cyc   wait/step {wt:8.1f} cyc")
for w in range(16):
    print(w, f"{st[:, w, 0].mean() / nsteps:8.1f} {st[:, w, 1].mean() / nsteps:8.1f}")
