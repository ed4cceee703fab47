"""In-tree build of libpsgla_hip.so (gfx950).  Used by ``__graft_entry__.build()``.

One translation unit per kernel family (csrc/*.hip), compiled in parallel, then linked:

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -I include \
          -c csrc/<unit>.hip -o build/<unit>.o          (one process per unit)
    hipcc -shared -fPIC -o psgla_for_posterior_sampling_amd/libpsgla_hip.so build/*.o

-fno-slp-vectorize: packed fp32 (v_pk_*) needs operand shuffles and measured slower on gfx950.
-ffp-contract=off keeps the reference's separate multiply/add roundings (the EXACT
kernels are bit-identical to the torch CPU checker); fmas are written explicitly
where the fast kernels want them.

tv_tile.hip adds -mllvm -amdgpu-sched-strategy=max-ilp (UNIT_FLAGS): the tile kernel is latency-bound at four
waves per SIMD, and the ILP-first machine scheduler measured -1.7 % at 8 chains and -0.7 % for castle at batch 1
(the row stream +0.3 %, so it keeps the default; profiles/r05s_sched_strategy_ab.txt).

Diagnostic variants (tools/variant_build.py) rebuild only the units their patches touch.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
UNITS = ["api", "tv_stream", "tv_tile", "tv_band", "blur", "elementwise"]
SOURCES = [os.path.join(CSRC, u + ".hip") for u in UNITS]
HEADERS = [os.path.join(CSRC, "noise.hpp"), os.path.join(CSRC, "psgla_common.hpp"),
           os.path.join(REPO, "include", "psgla_hip.h")]
OUT = os.path.join(PKG, "libpsgla_hip.so")
OBJ = os.path.join(REPO, "build", "obj")
ARCH = os.environ.get("PSGLA_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-Wno-inline-asm", "-fPIC"]
UNIT_FLAGS = {"tv_tile": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libpsgla_hip.so)")


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(s) <= t for s in SOURCES + HEADERS)


def compile_units(sources, objdir, extra=(), include=(), verbose=False):
    """Compile each source to objdir/<name>.o in parallel; returns the object paths."""
    os.makedirs(objdir, exist_ok=True)
    inc = ["-I", os.path.join(REPO, "include"), "-I", CSRC]
    for d in include:
        inc += ["-I", d]

    def one(src):
        obj = os.path.join(objdir, os.path.splitext(os.path.basename(src))[0] + ".o")
        unit = os.path.splitext(os.path.basename(src))[0]
        cmd = [hipcc(), f"--offload-arch={ARCH}"] + FLAGS + UNIT_FLAGS.get(unit, []) + list(extra) + inc + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    jobs = min(len(sources), max(1, int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        return list(ex.map(one, sources))


def link(objs, out, verbose=False):
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + list(objs)
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build_native(force: bool = False, verbose: bool = False, out: str = OUT) -> str:
    if not force and out == OUT and up_to_date():
        return OUT
    extra = os.environ.get("PSGLA_HIPCC_EXTRA", "").split()
    objs = compile_units(SOURCES, OBJ, extra=extra, verbose=verbose)
    return link(objs, out, verbose=verbose)


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
    print("units:", sorted(os.path.basename(p) for p in glob.glob(os.path.join(OBJ, "*.o"))))
