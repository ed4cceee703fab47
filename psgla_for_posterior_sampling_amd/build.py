"""In-tree build of libpsgla_hip.so (gfx950).  Used by ``__graft_entry__.build()``.

    hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared -I include \
          -o psgla_for_posterior_sampling_amd/libpsgla_hip.so csrc/psgla_kernels.hip

-fno-slp-vectorize: packed fp32 (v_pk_*) needs operand shuffles and measured slower on gfx950.
-ffp-contract=off keeps the reference's separate multiply/add roundings (the EXACT
kernels are bit-identical to the torch CPU checker); fmas are written explicitly
where the fast kernels want them.
"""
from __future__ import annotations

import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
SOURCES = [os.path.join(PKG, "csrc", "psgla_kernels.hip")]
HEADERS = [os.path.join(PKG, "csrc", "noise.hpp"), os.path.join(REPO, "include", "psgla_hip.h")]
OUT = os.path.join(PKG, "libpsgla_hip.so")
ARCH = os.environ.get("PSGLA_OFFLOAD_ARCH", "gfx950")


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


def build_native(force: bool = False, verbose: bool = False, out: str = OUT) -> str:
    if not force and out == OUT and up_to_date():
        return OUT
    extra = os.environ.get("PSGLA_HIPCC_EXTRA", "").split()
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-Wno-inline-asm", "-fPIC",
           "-shared", "-I", os.path.join(REPO, "include"), "-o", out + ".tmp"] + extra + SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_native(force=True, verbose=True))
