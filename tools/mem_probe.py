"""Times tools/mem_probe.hip (exp_libs/libmem_probe.so, built by tools/mem_probe.sh): the row-stream
pipeline's HBM access pattern without its arithmetic, at the bench shape (64 x 3 x 256 x 256).  Prints one
JSON line per variant: microseconds per launch and the algorithmic bytes moved / time."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(REPO, "exp_libs", "libmem_probe.so"))
P_, c_i32 = ctypes.c_void_p, ctypes.c_int32


class ProbeArgs(ctypes.Structure):
    _fields_ = [(n, P_) for n in ("x", "u2", "y", "mask", "mean", "sq", "xo", "u2o", "meano", "sqo")] + \
               [(n, c_i32) for n in ("P", "H", "W", "nwg", "halo", "lead", "depth", "order")]


def main():
    B, C, H, W = 64, 3, 256, 256
    dev = "cuda:0"
    f = dict(dtype=torch.float32, device=dev)
    t = {k: torch.rand((B, C, H, W), **f) for k in ("x", "y", "mean", "sq", "xo", "meano", "sqo")}
    t["u2"] = torch.rand((B, C, H, W, 2), **f)
    t["u2o"] = torch.rand((B, C, H, W, 2), **f)
    t["mask"] = (torch.rand((H, W), device=dev) > 0.5).to(torch.uint8)
    a = ProbeArgs()
    for k, v in t.items():
        setattr(a, k, v.data_ptr())
    a.P, a.H, a.W, a.halo, a.lead, a.depth = B * C, H, W, 10, 4, 34
    st = torch.cuda.current_stream()
    T = B * C * H

    def algo_bytes(nwg, halo):
        tot = 0
        for b in range(nwg):
            c0, c1 = T * b // nwg, T * (b + 1) // nwg
            l0, l1 = max(0, c0 - halo), min(T, c1 + halo)
            tot += (l1 - l0) * (W * 4 * 4 + W) + (c1 - c0) * W * 4 * 7
        return tot

    runs = [(0, 256, 0, 4), (1, 256, 0, 4), (2, 256, 0, 4), (0, 256, 1, 4), (0, 512, 0, 4), (3, 0, 0, 4)]
    if len(sys.argv) > 1:
        runs = [tuple(int(v) for v in r.split(",")) for r in sys.argv[1:]]
    for variant, nwg, order, lead in runs:
        a.nwg, a.order, a.lead = max(nwg, 8), order, lead
        grid = 256 * 8 if variant == 3 else 0
        for _ in range(200 if variant >= 4 else 20):
            assert lib.probe_launch(ctypes.byref(a), variant, grid, ctypes.c_void_p(st.cuda_stream)) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            lib.probe_launch(ctypes.byref(a), variant, grid, ctypes.c_void_p(st.cuda_stream))
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        byt = algo_bytes(a.nwg, 10) if variant != 3 else T * (W * 4 * 11 + W)
        print(json.dumps({"variant": variant, "nwg": a.nwg, "order": order, "lead": lead, "us": round(us, 2),
                          "MB": round(byt / 1e6, 1), "TBps": round(byt / us / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
