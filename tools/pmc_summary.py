"""Summarise rocprofv3 PMC passes of the fused-step kernel into profiles/<round>_pmc_<kernel>.json.

    python3 tools/pmc_summary.py --round r01 --kernel tv_stream_kernel gpurun_out/pmc1 gpurun_out/pmc2 ...

Each directory holds one `--pmc ... --output-format csv` pass (p_counter_collection.csv).
Counter values are summed over the per-XCD / per-SE rows of a dispatch and averaged over the
dispatches of the kernel.  HBM traffic per launch follows MI355X_MICROARCH.md's rocprofv3
section: FETCH_SIZE and WRITE_SIZE are in KiB, collected in separate passes, and FETCH_SIZE
is doubled on gfx950 (it tallies the 128-B requests of wide streaming reads at 64 B).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os


def load(dirs, kernel):
    per = collections.defaultdict(list)
    for d in dirs:
        path = os.path.join(d, "p_counter_collection.csv")
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            if kernel not in r["Kernel_Name"]:
                continue
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, c), v in agg.items():
            per[c].append(v)
    return {c: sum(v) / len(v) for c, v in per.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dirs", nargs="+")
    p.add_argument("--round", default="r01")
    p.add_argument("--kernel", default="tv_stream_kernel")
    p.add_argument("--out", default=None)
    p.add_argument("--commit", default=None, help="git commit the profiled tree was built from")
    p.add_argument("--chains", type=int, default=64, help="chains per GPU of the profiled bench run")
    p.add_argument("--exact", action="store_true", help="the profiled run used the exact kernel")
    p.add_argument("--command", default=None, help="the profiled command")
    a = p.parse_args()
    c = load(a.dirs, a.kernel)
    out = {"kernel": a.kernel, "counters_per_dispatch": c, "commit": a.commit, "exact": bool(a.exact),
           "workload": {"chains_per_gpu": a.chains, "image": [3, 256, 256], "n_tv": 10}, "command": a.command}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fetch = 2.0 * c["FETCH_SIZE"] * 1024.0
        write = c["WRITE_SIZE"] * 1024.0
        out["hbm_read_bytes_per_launch"] = fetch
        out["hbm_write_bytes_per_launch"] = write
        out["hbm_bytes_per_launch"] = fetch + write
        out["note"] = "FETCH_SIZE x2 (gfx950 correction), KiB -> bytes; separate passes"
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        out["wave_cycle_split"] = {k: c[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                          "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS") if k in c}
    path = a.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                 f"{a.round}_pmc_{a.kernel.replace('_kernel', '')}.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(path)
    print(json.dumps({k: v for k, v in out.items() if k != "counters_per_dispatch"}, indent=1))


if __name__ == "__main__":
    main()
