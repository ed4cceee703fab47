"""Compile one translation unit with -Rpass-analysis=kernel-resource-usage and print one line per kernel:
VGPRs, AGPRs, spills, scratch, occupancy.  Usage: python3 tools/kernel_resources.py csrc/tv_stream.hip [-Dflags]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from psgla_for_posterior_sampling_amd import build as B  # noqa: E402

src = sys.argv[1]
cmd = [B.hipcc(), f"--offload-arch={B.ARCH}"] + B.FLAGS + ["-I", os.path.join(REPO, "include"), "-I", B.CSRC,
                                                           "-I", os.path.dirname(os.path.abspath(src))] + \
    sys.argv[2:] + ["-c", src, "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True)
cur = None
rows = []
for line in out.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s*(\S+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
    elif "error" in line:
        print(line)
for r in rows:
    n = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    print(f"{n[:90]:90s} vgpr {r.get('VGPRs', '?'):>4s} agpr {r.get('AGPRs', '?'):>3s} "
          f"vspill {r.get('VGPRs Spill', '?'):>3s} sspill {r.get('SGPRs Spill', '?'):>4s} "
          f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4s} occ {r.get('Occupancy [waves/SIMD]', '?')}")
sys.exit(out.returncode)
