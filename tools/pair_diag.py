"""Per-role phase timing of the row-pair kernel from the diagnostic library (tools/pair_diag_source.py):
average shader cycles per step that each wave spends working / waiting in the W and C phases."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PSGLA_LIB", os.path.join(REPO, "exp_libs", "lib_diag.so"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psgla_for_posterior_sampling_amd import _native as N  # noqa: E402
from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402
from psgla_for_posterior_sampling_amd.engine import FusedTvChains  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
variant = sys.argv[2] if len(sys.argv) > 2 else "pair"
dev = torch.device("cuda:0")
xs = torch.rand((B, 3, 256, 256), device=dev)
mask2d = (torch.rand((256, 256), device=dev) > 0.5).to(torch.uint8)
y = mask2d.float() * xs
init = (mask2d.float() * y + (1 - mask2d.float()) * 0.5).contiguous()
eng = FusedTvChains(init, y.contiguous(), mask2d, c1=1.5e-4, c2=0.055, sigma2=1.5e-5, alpha=1.0, ths=0.039,
                    tv=K.TvConstants(n_it_max=10), seed=0, n_iter=400, n_inter=10, n_inter_mmse=10,
                    kernel_variant=variant)
eng.run(40, graph_steps=20)
torch.cuda.synchronize()
lib = N.lib()
lib.psgla_diag_set_buffer.argtypes = [ctypes.c_void_p]
grid = 256
buf = torch.zeros((grid, 16, 12), dtype=torch.int64, device=dev)
lib.psgla_diag_set_buffer(buf.data_ptr())
eng.launch_main_only(20)
torch.cuda.synchronize()
lib.psgla_diag_set_buffer(None)
d = buf.cpu().numpy().astype(np.float64)
steps = 129.0
roles = {"front": range(0, 4), "stage": range(4, 14), "back": range(14, 16)}
print(f"{variant} B={B}: cycles per step (avg over workgroups), W work / W wait / C work / C wait")
for name, ws in roles.items():
    for w in ws:
        v = d[:, w, :].mean(0) / steps
        print(f"  {name:5s} w{w:2d}: W {v[0]:7.0f} / {v[1]:7.0f}   C {v[2]:7.0f} / {v[3]:7.0f}")
for w in range(4):
    v = d[:, w, :].mean(0) / (steps / 4)
    print(f"  front w{w} per-phs work, W: " + " ".join(f"{x:6.0f}" for x in v[8:12]) + "   C: " + " ".join(f"{x:6.0f}" for x in v[4:8]))
for w in (14, 15):
    v = d[:, w, :].mean(0) / (steps / 2)
    print(f"  back w{w}: W (take / other) {v[8]:6.0f} {v[9]:6.0f}   C (take / other) {v[4]:6.0f} {v[5]:6.0f}")
tot = d[:, 0, :4].mean(0).sum() / steps
print(f"  step total (wave 0) {tot:.0f} cycles")
