"""Build a diagnostic variant of the product kernels from a patched copy of csrc/psgla_kernels.hip
(never loaded by the product: bench.py / tests pick it via PSGLA_LIB).  Each patch is an exact
(old, new, count) text replacement; the build fails if a pattern does not match.
Usage: python3 tools/variant_build.py NAME PATCHES.py   (PATCHES.py defines PATCHES = [(old, new, count), ...])"""
import os
import runpy
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name, patch_file = sys.argv[1], sys.argv[2]
src = open(os.path.join(REPO, "psgla_for_posterior_sampling_amd", "csrc", "psgla_kernels.hip")).read()
for old, new, count in runpy.run_path(patch_file)["PATCHES"]:
    if src.count(old) != count:
        raise SystemExit(f"pattern count {src.count(old)} != {count}: {old[:80]!r}")
    src = src.replace(old, new)
os.makedirs(os.path.join(REPO, "exp_libs", "src"), exist_ok=True)
path = os.path.join(REPO, "exp_libs", "src", f"{name}.hip")
open(path, "w").write(src)
csrc = os.path.join(REPO, "psgla_for_posterior_sampling_amd", "csrc")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
       "-Wno-inline-asm", "-fPIC", "-shared", "-I", os.path.join(REPO, "include"), "-I", csrc,
       "-o", os.path.join(REPO, "exp_libs", f"lib_{name}.so"), path]
subprocess.run(cmd, check=True)
print("built exp_libs/lib_%s.so" % name)
