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
NTV = int(os.environ.get("NTV", "10"))
g = torch.Generator(device=dev).manual_seed(1234)
xs = torch.rand((B, C, H, W), generator=g, device=dev)
gen = torch.Generator(device=dev).manual_seed(0)
mask_2d = 1 * (torch.rand((H, W), generator=gen, device=dev) > 0.5)
y = mask_2d * xs
init = mask_2d * y + (1 - mask_2d) * 0.5
s = 10 / 255.0
eng = FusedTvChains(init.contiguous().float(), y.contiguous().float(), mask_2d.to(torch.uint8), c1=1.5379e-4 * 10 / 10,
                    c2=0.0554594, sigma2=float(np.float32((1 / 255.0) ** 2)), alpha=1.0, ths=float(np.float32(s)),
                    tv=K.TvConstants(n_it_max=NTV), seed=0, n_iter=10, n_inter=10, n_inter_mmse=10,
                    stream_wgs=-1)
nsteps = H + 4 + 3 * NTV
stamps = torch.zeros((B * C * 32 + nsteps * 32 + B * C * 16,), dtype=torch.int64, device=dev)
eng.desc.debug_stamps = stamps.data_ptr()
eng.step(5)
torch.cuda.synchronize()
allst = stamps.cpu().numpy().astype(np.float64)
st = allst[:B * C * 32].reshape(B * C, 16, 2)
tr = allst[B * C * 32:B * C * 32 + nsteps * 32].reshape(nsteps, 16, 2)
segs = allst[B * C * 32 + nsteps * 32:].reshape(B * C, 4, 4)
roles = {"front": range(0, 4), "stage": range(4, 4 + NTV), "back": range(4 + NTV, 6 + NTV)}
for name, ws in roles.items():
    wk = st[:, list(ws), 0].mean() / nsteps
    wt = st[:, list(ws), 1].mean() / nsteps
    print(f"{name:6s} work/step {wk:8.1f} cyc   wait/step {wt:8.1f} cyc")
for w in range(6 + NTV):
    print(w, f"{st[:, w, 0].mean() / nsteps:8.1f} {st[:, w, 1].mean() / nsteps:8.1f}")

# workgroup 0 per-step trace: arrival (t1) and release (t0) of every wave
rel = tr[:, :, 1].max(axis=1)            # release time of step t (all waves see ~the same)
arr = tr[:, :, 0]
dur = np.diff(rel)
print("wg0 step duration: mean %.1f  median %.1f  p90 %.1f" % (dur.mean(), np.median(dur), np.percentile(dur, 90)))
a_rel = arr[1:] - rel[:-1, None]          # arrival after previous release
last = a_rel.argmax(axis=1)
print("last arriver histogram:", np.bincount(last, minlength=16))
print("mean arrival after release per wave:", a_rel.mean(axis=0).round(0))
print("barrier latency (release - last arrival): mean %.1f" % (rel[1:] - arr[1:].max(axis=1)).mean())
mid = slice(40, nsteps - 40)
print("steady-state (steps 40..-40): duration mean %.1f; mean arrival per wave:" % dur[mid].mean(), a_rel[mid].mean(axis=0).round(0))
# front waves: arrival by pipeline phase p = (t + 4 - fw) & 3 (0 Philox, 1/2 Box-Muller, 3 data term)
for fw in range(4):
    ph = [[] for _ in range(4)]
    for t in range(40, nsteps - 40):
        ph[(t + 4 - fw) & 3].append(a_rel[t - 1, fw])
    print("front", fw, "arrival by phase:", [round(float(np.mean(x)), 0) for x in ph])
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.save(os.path.join(REPO, "gpurun_out", "stamps_trace.npy"), tr)
print("front p3 segments per row (dma wait, compute, ring writes+lgkm, dma issue):", (segs.mean(axis=(0, 1)) / (H / 4)).round(1))
