"""The reference's per-image workload on the MI355X: PSGLA + TV on set1c castle (3 x 481 x 321, batch 1),
inpainting 50 %, the N = 10000 schedule of BASELINE configs[1] (n_inter = n_inter_mmse = 10): per-step time
of the fused step (graph replay) and the resulting PSNR_MMSE.  One JSON line on stdout."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402
from psgla_for_posterior_sampling_amd import metrics  # noqa: E402
from psgla_for_posterior_sampling_amd import sampling_images as SI  # noqa: E402
from psgla_for_posterior_sampling_amd.engine import FusedTvChains  # noqa: E402
from psgla_for_posterior_sampling_amd.fidelity import inpainting_problem  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
TRANSPOSE = len(sys.argv) > 3 and sys.argv[3] == "T"     # the other orientation (3 x 321 x 481: W = 481)
dev = torch.device("cuda:0")
im = np.float32(SI.read_image(os.path.join(REPO, "tests", "golden", "set1c", "castle.png")) / 255.)
if TRANSPOSE:
    im = np.ascontiguousarray(np.transpose(im, (1, 0, 2)))
im_t = torch.from_numpy(np.transpose(im, (2, 0, 1))).float().unsqueeze(0).to(dev)
dg, y, init, mask2d, _ = inpainting_problem(im_t, seed_ip=0)
s, lam = 10 / 255.0, 10.0
c1 = float((torch.tensor(s ** 2).float() / torch.tensor(lam).float()).item())
c2 = float((torch.tensor(np.sqrt(2)).float() * torch.tensor(s).float()).item())
eng = FusedTvChains(init.expand(B, -1, -1, -1).contiguous(), y, dg.mask_u8, c1=c1, c2=c2, sigma2=dg.sigma2,
                    alpha=1.0, ths=float(np.float32(s)), tv=K.TvConstants(n_it_max=10), seed=0, n_iter=N,
                    n_inter=max(1, N // 1000), n_inter_mmse=max(1, N // 1000))
eng.run(100, graph_steps=50)
torch.cuda.synchronize()
t0 = time.perf_counter()
eng.run(N - 100, graph_steps=50)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
Xl, Ml, M2l = eng.lists()
rec, _ = metrics.analyse_run(im, [x[0] if B > 1 else x for x in Xl[-3:]], [m[0] if B > 1 else m for m in Ml],
                             [m[0] if B > 1 else m for m in M2l], y, init)
Hc, Wc = im.shape[0], im.shape[1]
# roofline fraction of the fused step: compulsory bytes per launch (bench.algorithmic_bytes_per_launch, this run's
# schedule) / the per-step time / 8 TB/s
sys.path.insert(0, REPO)
from bench import algorithmic_bytes_per_launch  # noqa: E402
nb = algorithmic_bytes_per_launch(B, 3, Hc, Wc, 100, N - 100, max(1, N // 1000), max(1, N // 1000))
frac = nb / (dt / (N - 100)) / 8e12
print(json.dumps({"workload": f"psgla+TV inpainting, set1c castle 3x{Hc}x{Wc}", "chains": B, "n_iter": N,
                  "kernel": eng.main_kernel, "ms_per_step": round(dt / (N - 100) * 1e3, 5),
                  "image_steps_per_s": round(B * (N - 100) / dt, 1), "PSNR_MMSE": round(rec["PSNR_MMSE"], 3),
                  "PSNR_y": round(rec["PSNR_y"], 3), "blocks": len(Ml),
                  "algorithmic_bytes_per_step": round(nb), "roofline_frac": round(frac, 4)}))
