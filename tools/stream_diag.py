"""Per-role step timing of the row-stream kernel from its diagnostic library (tools/stream_diag_source.py)."""
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
lib.psgla_diag_set_buffer.argtypes = [ctypes.c_void_p]
buf = torch.zeros((256, 16, 8), dtype=torch.int64, device=dev)
lib.psgla_diag_set_buffer(buf.data_ptr())
eng.launch_main_only(20)
torch.cuda.synchronize()
lib.psgla_diag_set_buffer(None)
d = buf.cpu().numpy().astype(np.float64)
steps = 246.0
print(f"stream B={B}: cycles per step (avg over workgroups): work / wait")
for w in range(16):
    v = d[:, w, :].mean(0) / steps
    extra = ("   per-phase work: " + " ".join(f"{x * 4:6.0f}" for x in v[2:6])) if w < 4 else ""
    print(f"  w{w:2d}: {v[0]:7.0f} / {v[1]:7.0f}{extra}")
