"""Per-step barrier accounting of the row-stream kernel from the diagnostic library built by
`python3 tools/variant_build.py sdiag tools/patches/stream_stepdiag.py` (exp_libs/lib_sdiag.so).
Prints, averaged over workgroups 0..63 of one bench-shape launch: the step length, each wave's work (its
arrival - its release), and how often each wave is the last to arrive.  Usage: PSGLA_LIB=exp_libs/lib_sdiag.so python3 tools/stream_stepdiag.py [B]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PSGLA_LIB", os.path.join(REPO, "exp_libs", "lib_sdiag.so"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psgla_for_posterior_sampling_amd import _native as N  # noqa: E402
from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402
from psgla_for_posterior_sampling_amd.engine import FusedTvChains  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda:0")
xs = torch.rand((B, 3, 256, 256), device=dev)
mask2d = (torch.rand((256, 256), device=dev) > 0.5).to(torch.uint8)
y = mask2d.float() * xs
init = (mask2d.float() * y + (1 - mask2d.float()) * 0.5).contiguous()
eng = FusedTvChains(init, y.contiguous(), mask2d, c1=1.5e-4, c2=0.055, sigma2=1.5e-5, alpha=1.0, ths=0.039,
                    tv=K.TvConstants(n_it_max=10), seed=0, n_iter=400, n_inter=10, n_inter_mmse=10,
                    kernel_variant="stream")
eng.run(40, graph_steps=20)
torch.cuda.synchronize()
lib = N.lib()
lib.psgla_stepdiag_set_buffer.argtypes = [ctypes.c_void_p]
lib.psgla_stepdiag_set_buffer.restype = ctypes.c_int
buf = torch.zeros((64, 64), dtype=torch.int64, device=dev)
assert lib.psgla_stepdiag_set_buffer(buf.data_ptr()) == 0
eng.launch_main_only(3)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
eng.launch_main_only(1)
ev1.record()
torch.cuda.synchronize()
ms = ev0.elapsed_time(ev1)
lib.psgla_stepdiag_set_buffer(None)
d = buf.cpu().numpy().astype(np.float64)
n = d[:, 0]
per = lambda col: (d[:, col] / n).mean()  # noqa: E731
print(f"stream B={B}: launch {ms*1e3:.1f} us (diag build); steps per workgroup {n.mean():.1f}")
print(f"  per step (s_memtime ticks): length {per(1):.0f}")
roles = ["front"] * 4 + [f"stage{k}" for k in range(1, 11)] + ["back"] * 2
if os.environ.get("PSGLA_STREAM_LAYOUT") == "2":     # the merged layout of commit 8674423 (12 waves)
    roles = ["front"] * 4 + ["st1+2", "st3+4", "st5+6", "st7+8", "stage9", "stage10"] + ["back"] * 2 + ["-"] * 4
for w in range(16):
    print(f"  w{w:2d} {roles[w]:>7s}: work {per(4 + w):6.0f}   last to arrive in {100 * (d[:, 20 + w] / n).mean():5.1f} % of steps")
