"""A/B of two builds of the deblurring stencil (diagnostic): run under PSGLA_LIB=<lib> with a tag, then
`python tools/blur_ab.py --compare TAG1 TAG2` checks the saved outputs for bitwise equality.

    PSGLA_LIB=exp_libs/lib_X.so python tools/blur_ab.py --tag X
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

CASES = [  # B, H, W, l
    (2, 40, 52, 4), (1, 37, 29, 4), (2, 70, 130, 2), (1, 16, 16, 0), (1, 64, 64, 1), (1, 45, 70, 3),
    (1, 100, 90, 5), (1, 50, 44, 8), (2, 256, 256, 4), (1, 321, 481, 4), (1, 481, 321, 7), (1, 33, 40, 6),
]


def taps(l):
    h = np.ones((1, 2 * l + 1))
    h = np.exp(-((np.arange(-l, l + 1) / 1.3) ** 2))[None] * h
    h = h / h.sum()
    h_ = h.T @ h
    return torch.from_numpy(np.flip(h_).copy()).float(), torch.from_numpy(h_).float()


def run(tag, no_sep=False):
    from psgla_for_posterior_sampling_amd import hip_ops as K
    if no_sep:
        K.blur_set_separable(False)
    dev = "cuda"
    out = {}
    g = torch.Generator().manual_seed(0)
    for (B, H, W, l) in CASES:
        x = torch.rand((B, 3, H, W), generator=g).to(dev)
        y = torch.rand((B, 3, H, W), generator=g).to(dev)
        hc, hr = taps(l)
        s2 = float(np.float32((1 / 255.0) ** 2))
        for exact in (True, False):
            out[str((B, H, W, l, exact, "g"))] = K.blur_grad(x, y, hc, hr, l, s2, exact=exact).cpu()
            out[str((B, H, W, l, exact, "Y"))] = K.blur_langevin(x, y, hc, hr, l, s2, 1e-4, 0.05, seed=5, chain0=1,
                                                            step=3, exact=exact).cpu()
    torch.save(out, f"gpurun_out/blur_{tag}.pt")
    # timing at the config-4 shape: 64 x 3 x 256 x 256, l = 4
    B, H, W, l = 64, 3, 256, 4
    X = torch.rand((64, 3, 256, 256), device=dev)
    Y = torch.rand((64, 3, 256, 256), device=dev)
    o = torch.empty_like(X)
    hc, hr = taps(4)
    s2 = float(np.float32((1 / 255.0) ** 2))
    E = X.numel()
    for exact in (False, True):
        for name, fn in (("grad", lambda: K.blur_grad(X, Y, hc, hr, 4, s2, out=o, exact=exact)),
                         ("langevin", lambda: K.blur_langevin(X, Y, hc, hr, 4, s2, 1e-4, 0.05, 0, 0, 5, out=o,
                                                              exact=exact))):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            fl = 2 * 2 * 81 * E
            print(f"{tag:>10s} {name:9s} exact={int(exact)} {ms * 1e3:8.1f} us  {fl / ms / 1e9:6.1f} TFLOP/s "
                  f"(2 x 81 MAC / elem)  {12 * E / ms / 1e9:6.2f} TB/s", flush=True)


def compare(t1, t2):
    a = torch.load(f"gpurun_out/blur_{t1}.pt", weights_only=True)
    b = torch.load(f"gpurun_out/blur_{t2}.pt", weights_only=True)
    bad = 0
    for k in a:
        same = torch.equal(a[k], b[k])
        if not same:
            bad += 1
            d = (a[k] - b[k]).abs().max().item()
            print("DIFF", k, f"max|d| {d:.3e}  max|a| {a[k].abs().max().item():.3e}  rel {d / a[k].abs().max().item():.2e}")
    print(f"{len(a) - bad}/{len(a)} outputs bitwise equal")
    return bad


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--tag")
    p.add_argument("--compare", nargs=2)
    p.add_argument("--no-sep", action="store_true", help="fast mode on the 2-D stencil (psgla_blur_set_separable(0))")
    a = p.parse_args()
    if a.compare:
        sys.exit(1 if compare(*a.compare) else 0)
    run(a.tag, a.no_sep)
