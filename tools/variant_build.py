"""Build a diagnostic variant of the product library from patched copies of csrc/*.hip (never loaded by the
product: bench.py / tests pick it via PSGLA_LIB).  Each patch is an exact (old, new, count) text replacement
searched over every translation unit (and psgla_common.hpp); the build fails if a pattern's total count
differs.  Only the units whose text changed are recompiled -- the others reuse the product objects in
build/obj (run ``python -m psgla_for_posterior_sampling_amd.build`` first); a changed header recompiles all.
Usage: python3 tools/variant_build.py NAME PATCHES.py [NAME2 PATCHES2.py ...]
       (PATCHES.py defines PATCHES = [(old, new, count), ...]; extra hipcc flags: EXTRA = ["-D...", ...];
        FORCE = ["tv_stream.hip", ...] recompiles those units from the working tree even if no patch touches them;
        SOURCE_OVERRIDE = {"tv_stream.hip": "/path/file.hip"} takes a unit's text from another file, e.g. a
        committed version, before the patches apply)"""
import os
import runpy
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from psgla_for_posterior_sampling_amd import build as B  # noqa: E402


def variant(name, patch_file):
    spec = runpy.run_path(patch_file)
    files = {os.path.basename(p): open(p).read() for p in B.SOURCES + [os.path.join(B.CSRC, "psgla_common.hpp")]}
    orig = dict(files)
    for unit, path in spec.get("SOURCE_OVERRIDE", {}).items():   # e.g. a unit as committed (git show) as the base
        files[unit] = open(path).read()
    for old, new, count in spec.get("PATCHES", []):
        total = sum(t.count(old) for t in files.values())
        if total != count:
            raise SystemExit(f"{name}: pattern count {total} != {count}: {old[:80]!r}")
        files = {k: t.replace(old, new) for k, t in files.items()}
    src_dir = os.path.join(REPO, "exp_libs", "src", name)
    obj_dir = os.path.join(REPO, "exp_libs", "obj", name)
    if os.path.isdir(src_dir):
        shutil.rmtree(src_dir)
    os.makedirs(src_dir)
    for k, t in files.items():
        open(os.path.join(src_dir, k), "w").write(t)
    shutil.copy(os.path.join(B.CSRC, "noise.hpp"), src_dir)
    extra = list(spec.get("EXTRA", []))
    changed = [k for k in files if files[k] != orig[k]] + list(spec.get("FORCE", []))
    rebuild_all = "psgla_common.hpp" in changed or extra
    units = [os.path.join(src_dir, os.path.basename(s)) for s in B.SOURCES
             if rebuild_all or os.path.basename(s) in changed]
    objs = {os.path.basename(o): o for o in B.compile_units(units, obj_dir, extra=extra, include=[src_dir])} if units else {}
    link = []
    for s in B.SOURCES:
        o = os.path.splitext(os.path.basename(s))[0] + ".o"
        link.append(objs.get(o, os.path.join(B.OBJ, o)))
    out = os.path.join(REPO, "exp_libs", f"lib_{name}.so")
    B.link(link, out)
    print(f"built exp_libs/lib_{name}.so (recompiled: {', '.join(os.path.basename(u) for u in units) or 'none'})")


if __name__ == "__main__":
    args = sys.argv[1:]
    if not args or len(args) % 2:
        raise SystemExit(__doc__)
    for i in range(0, len(args), 2):
        variant(args[i], args[i + 1])
