"""Per-phase budget of one tv_tile_kernel launch (the strong-scaling kernel) from the diagnostic library built by
`python3 tools/variant_build.py tdiag tools/patches/tile_phasediag.py` (exp_libs/lib_tdiag.so).
Replays 20-step graph segments of the fused step at B chains of 3 x H x W and reads the stamps of the last two
launches (100 MHz real-time counter, common to all CUs): per workgroup the kernel entry, loads issued + noise, loads
landed + data term, inner iterations, rel-err / X side / u2 issued, arrival, and the last workgroup's finalisation.
Prints the launch's critical path, the per-phase means over workgroups and the gap between two launches.
Usage: PSGLA_LIB=exp_libs/lib_tdiag.so python3 tools/tile_phasediag.py [B] [H] [W]"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PSGLA_LIB", os.path.join(REPO, "exp_libs", "lib_tdiag.so"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from psgla_for_posterior_sampling_amd import _native as N  # noqa: E402
from psgla_for_posterior_sampling_amd import hip_ops as K  # noqa: E402
from psgla_for_posterior_sampling_amd.engine import FusedTvChains  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
H = int(sys.argv[2]) if len(sys.argv) > 2 else 256
W = int(sys.argv[3]) if len(sys.argv) > 3 else 256
dev = torch.device("cuda:0")
torch.manual_seed(0)
xs = torch.rand((B, 3, H, W), device=dev)
mask2d = (torch.rand((H, W), device=dev) > 0.5).to(torch.uint8)
y = mask2d.float() * xs
init = (mask2d.float() * y + (1 - mask2d.float()) * 0.5).contiguous()
eng = FusedTvChains(init, y.contiguous(), mask2d, c1=1.5e-4, c2=0.055, sigma2=1.5e-5, alpha=1.0, ths=0.039,
                    tv=K.TvConstants(n_it_max=10), seed=0, n_iter=4000, n_inter=10, n_inter_mmse=10,
                    kernel_variant="tile")
eng.run(200, graph_steps=20)                     # warm-up (graph captured)
torch.cuda.synchronize()
lib = N.lib()
lib.psgla_tilediag_set_buffer.argtypes = [ctypes.c_void_p]
lib.psgla_tilediag_set_buffer.restype = ctypes.c_int
buf = torch.zeros((2, 4096, 8), dtype=torch.int64, device=dev)
assert lib.psgla_tilediag_set_buffer(buf.data_ptr()) == 0
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
eng.run(20, graph_steps=20)
ev1.record()
torch.cuda.synchronize()
lib.psgla_tilediag_set_buffer(None)
ms = ev0.elapsed_time(ev1) / 20
d = buf.cpu().numpy().astype(np.float64)
G = int((d[0, :, 0] > 0).sum())
assert G == int((d[1, :, 0] > 0).sum()) and G > 0, "both slots must hold one launch"
later = 0 if d[0, :G, 0].min() > d[1, :G, 0].min() else 1
A, Bq = d[1 - later, :G], d[later, :G]          # launch k - 1, launch k (10 ns ticks)
us = lambda t: t / 100.0  # noqa: E731


def budget(L):
    t0 = L[:, 0].min()
    work = L[:, 1] > 0                          # workgroups that ran a tile (the rest only arrive)
    # the finalising workgroup: its stamp 6 lies in this launch (a stale 6 of another launch is older than t0)
    fin = np.where(L[:, 6] >= L[:, 5].max() - 1)[0] if (L[:, 6] >= t0).any() else np.array([], dtype=int)
    fin = int(fin[np.argmax(L[fin, 6])]) if fin.size else int(np.argmax(L[:, 5]))
    end = max(L[fin, 6], L[:, 5].max())
    ph = {
        "dispatch_spread": us(L[:, 0].max() - t0),
        "issue_noise": us((L[work, 1] - L[work, 0]).mean()),
        "loads_data_term": us((L[work, 2] - L[work, 1]).mean()),
        "iterations": us((L[work, 3] - L[work, 2]).mean()),
        "relerr_x_u2_issue": us((L[work, 4] - L[work, 3]).mean()),
        "store_drain_arrive": us((L[work, 5] - L[work, 4]).mean()),
        "finalise": us(L[fin, 6] - L[fin, 5]),
        "span": us(end - t0),
        "arrival_spread": us(L[:, 5].max() - L[:, 5].min()),
        "mean_workgroup_span": us((L[work, 5] - L[work, 0]).mean()),
    }
    return ph, end


if os.environ.get("TDIAG_CLOCK"):                # tools/patches/tile_clock.py: shader ticks over the iterations
    for L, nm in ((A, "launch_k-1"), (Bq, "launch_k")):
        work = L[:, 1] > 0
        ghz = L[work, 7] / ((L[work, 3] - L[work, 2]) * 10.0)
        print(f"shader clock over the iterations ({nm}): mean {ghz.mean():.3f} GHz, min {ghz.min():.3f}, max {ghz.max():.3f}")
if os.environ.get("TDIAG_FIN7"):                 # tools/patches/tile_fin_stamp.py: stamp 7 after the norms exchange
    for L, nm in ((A, "launch_k-1"), (Bq, "launch_k")):
        fin = int(np.argmax(L[:, 6]))
        print(f"finaliser ({nm}): arrival -> norms read {us(L[fin, 7] - L[fin, 5]):.2f} us, "
              f"-> end {us(L[fin, 6] - L[fin, 7]):.2f} us")
if os.environ.get("TDIAG_NUNC"):                 # tools/patches/tile_nuncert.py: tiles leaving a stop possible
    for L, nm in ((A, "launch_k-1"), (Bq, "launch_k")):
        fin = int(np.argmax(L[:, 6]))
        print(f"finaliser ({nm}): {int(L[fin, 7])} of {G} tiles leave a stop possible")
pa, endA = budget(A)
pb, _ = budget(Bq)
gap = us(Bq[:, 0].min() - endA)
out = {"B": B, "H": H, "W": W, "workgroups": G, "ms_per_step_events": round(ms, 5),
       "launch_k": {k: round(v, 2) for k, v in pb.items()}, "launch_k-1": {k: round(v, 2) for k, v in pa.items()},
       "gap_between_launches_us": round(gap, 2)}
print(json.dumps(out))
print(f"tile B={B} {H}x{W}: {G} workgroups, {ms * 1e3:.1f} us per step (events, diag build)")
for k in pb:
    print(f"  {k:>20s}: {pb[k]:7.2f} us   (previous launch {pa[k]:7.2f})")
print(f"  {'gap to next launch':>20s}: {gap:7.2f} us")

# Per-workgroup view of launch k (why the arrival spread): phase durations of the earliest and the latest arrivals,
# the arrival spread per XCD (workgroups x and x + 8 share one) and the correlation of the arrival with each phase
if os.environ.get("TDIAG_WG"):
    L = Bq
    t0 = L[:, 0].min()
    work = np.where(L[:, 1] > 0)[0]
    arr = us(L[work, 5] - t0)
    cols = ["entry", "issue_noise", "loads", "iterations", "relerr_u2", "drain_arrive"]
    ph = np.stack([us(L[work, 0] - t0)] + [us(L[work, i + 1] - L[work, i]) for i in range(5)], axis=1)
    order = np.argsort(arr)
    print("  per-workgroup phases (us): blockIdx | xcd | " + " | ".join(cols) + " | arrival")
    for sel, name in ((order[:6], "earliest"), (order[-6:], "latest")):
        print(f"  -- {name}")
        for i in sel:
            print("   %5d | %d | " % (work[i], work[i] & 7) + " | ".join(f"{v:6.2f}" for v in ph[i]) + f" | {arr[i]:6.2f}")
    for x in range(8):
        m = (work & 7) == x
        if m.any():
            print(f"  xcd {x}: {m.sum():3d} wgs, arrival {arr[m].min():6.2f} .. {arr[m].max():6.2f} us, mean {arr[m].mean():6.2f}")
    for j, c in enumerate(cols):
        if ph[:, j].std() > 0:
            print(f"  corr(arrival, {c:>12s}) = {np.corrcoef(arr, ph[:, j])[0, 1]:+.2f}   std {ph[:, j].std():5.2f} us")
