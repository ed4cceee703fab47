"""One main-pass-only launch of the row stream (no finalisation) with the barrier-count diagnostic library
(tools/patches/bar_count.py); prints each workgroup's per-wave barrier counts when they differ.
Usage: PSGLA_LIB=exp_libs/lib_barc.so python3 tools/bar_probe.py [B H W]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from psgla_for_posterior_sampling_amd import _native as N  # noqa: E402
from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402
from psgla_for_posterior_sampling_amd.engine import FusedTvChains  # noqa: E402

B, H, W = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (4, 48, 64)))
dev = torch.device("cuda:0")
lib = N.lib()
lib.psgla_barcount_set.argtypes = [ctypes.c_void_p]
buf = torch.zeros(4096 * 16, dtype=torch.int32, device=dev)
assert lib.psgla_barcount_set(buf.data_ptr()) == 0
g = torch.Generator(device=dev).manual_seed(5)
xs = torch.rand((B, 3, H, W), generator=g, device=dev)
mask2d = (torch.rand((H, W), generator=g, device=dev) > 0.5).to(torch.uint8)
y = mask2d.float() * xs
init = (mask2d.float() * y + (1 - mask2d.float()) * 0.5).contiguous()
eng = FusedTvChains(init, y.contiguous(), mask2d, c1=1.5e-4, c2=0.055, sigma2=1.5e-5, alpha=1.0, ths=0.039,
                    tv=K.TvConstants(n_it_max=10), seed=0, n_iter=8, n_inter=5, n_inter_mmse=4, kernel_variant="stream")
print("kernel", eng.main_kernel, flush=True)
eng.launch_main_only(1)
torch.cuda.synchronize()
c = buf.view(-1, 16).cpu()
nwg = int((c.sum(1) > 0).sum().item())
bad = 0
for wg in range(nwg):
    row = c[wg].tolist()
    if len(set(row)) > 1:
        bad += 1
        if bad <= 10:
            print("wg", wg, row)
print(f"{nwg} workgroups, {bad} with unequal per-wave barrier counts", flush=True)
