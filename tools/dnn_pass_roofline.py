#!/usr/bin/env python3
"""Achieved HBM bandwidth of the DNN configurations' HIP passes from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --stats --output-format csv -d D -o p -- python3 tools/bench_dnn.py --workload W ...
    python3 tools/dnn_pass_roofline.py --workload W --stats D/.../p_kernel_stats.csv [--batch 64 --H 256 --W 256]

Per pass: the average launch duration from the trace's kernel statistics (rocprofv3's own clock, not a
subtraction of wall times) and its algorithmic bytes per launch, SURVEY.md section 8(d):

* V-DnCNN, inpainting (`relax_langevin_inpaint_kernel`, restoration_algorithms.py:238-271 + :232-236 of the next
  step): read D 4 + y 4 (+ mean 4 + sq 4 except at a block start), write Y' 4 + mean 4 + sq 4 (the block means at a
  block end), + the sample 4 every n_inter steps, + the shared (H, W) u8 mask: 28.33 B/elem at the bench schedule;
* deblurring (two passes): `relax_accumulate_kernel` read Y 4 + D 4 (+ 8), write X 4 + 8 (+ sample), and the
  stencil kernel with the Langevin update fused (`blur_sep_kernel` / `blur_grad_kernel`): read X 4 + y 4, write
  Y' 4 (the stencil's halo re-reads are not algorithmic);
* V-ULA (`pnpula_prior_update_kernel`, restoration_algorithms.py:104-144 with sampling_images.py:156-157): read X 4
  + D 4 + y 4 (+ 8), write X' 4 + 8 (+ sample), + the mask: 32.33 B/elem.

The accumulator terms are averaged over the schedule (n_inter, n_inter_mmse) of tools/bench_dnn.py."""
from __future__ import annotations

import argparse
import csv
import json

PEAK_GBS = 8000.0


def acc_bytes(nm: int, n_inter: int) -> float:
    """Accumulator / sample bytes per element, averaged over a schedule: mean + sq written every step, read except
    at a block start (1 step in nm + 1), the sample every n_inter steps."""
    return 8.0 + 8.0 * nm / (nm + 1) + 4.0 / n_inter


def passes(workload: str, E: int, HW: int, nm: int, n_inter: int):
    a = acc_bytes(nm, n_inter)
    if workload == "dncnn-inpaint":
        return {"relax_langevin_inpaint_kernel": (4 + 4 + 4 + a) * E + HW}
    if workload == "dncnn-deblur":
        return {"relax_accumulate_kernel": (4 + 4 + 4 + a) * E, "blur_sep_kernel": 12.0 * E,
                "blur_grad_kernel": 12.0 * E}
    if workload == "drunet-ula":
        return {"pnpula_prior_update_kernel": (4 + 4 + 4 + 4 + a) * E + HW}
    raise ValueError(workload)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", required=True, choices=["dncnn-inpaint", "dncnn-deblur", "drunet-ula"])
    p.add_argument("--stats", required=True, help="rocprofv3 p_kernel_stats.csv")
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--C", type=int, default=3)
    p.add_argument("--H", type=int, default=256)
    p.add_argument("--W", type=int, default=256)
    a = p.parse_args()
    nm, n_inter = (10, 10) if a.workload.startswith("dncnn") else (1000, 1000)
    E = a.batch * a.C * a.H * a.W
    want = passes(a.workload, E, a.H * a.W, nm, n_inter)
    rows = list(csv.DictReader(open(a.stats)))
    total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    out = {"workload": a.workload, "chains": a.batch, "image": [a.C, a.H, a.W], "schedule": {"n_inter": n_inter,
           "n_inter_mmse": nm}, "stats": a.stats, "passes": []}
    for r in rows:
        name = r["Name"]
        for k, nbytes in want.items():
            if k in name:
                avg_ns = float(r["AverageNs"])
                gbs = nbytes / (avg_ns * 1e-9) / 1e9
                out["passes"].append({"kernel": name, "calls": int(r["Calls"]), "avg_us": round(avg_ns / 1e3, 2),
                                      "algorithmic_bytes": int(nbytes), "bytes_per_elem": round(nbytes / E, 3),
                                      "achieved_gbs": round(gbs, 1), "frac_of_8tbs": round(gbs / PEAK_GBS, 3),
                                      "share_of_gpu_time": round(float(r["TotalDurationNs"]) / total_ns, 4)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
