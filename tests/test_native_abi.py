"""CPU-side checks of the C-ABI library: it loads without a GPU, exports every entry point
declared in include/psgla_hip.h, and the ctypes descriptor layouts match the C structs."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "psgla_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_entry_points():
    fns = declared_functions()
    for f in ("psgla_tv_step", "psgla_tv_prox", "psgla_langevin_update", "psgla_relax_accumulate",
              "pnpula_update", "psgla_normal_fill", "psgla_inpaint_grad", "psgla_abi_version"):
        assert f in fns


def test_library_loads_and_exports_every_declared_symbol():
    from psgla_for_posterior_sampling_amd import _native as N
    lib = N.lib()
    for f in declared_functions():
        assert hasattr(lib, f), f
        assert f in N.EXPORTED_SYMBOLS, f"{f} not bound in _native"
    assert lib.psgla_abi_version() == N.ABI_VERSION


def test_struct_layouts_match_c(tmp_path):
    from psgla_for_posterior_sampling_amd import _native as N
    prog = tmp_path / "sz.c"
    fields = {"PsglaTvStep": [f[0] for f in N.PsglaTvStep._fields_],
              "PsglaSchedule": [f[0] for f in N.PsglaSchedule._fields_],
              "PsglaTvProx": [f[0] for f in N.PsglaTvProx._fields_]}
    lines = ['#include "psgla_hip.h"', "#include <stdio.h>", "#include <stddef.h>", "int main(void){"]
    for s, fs in fields.items():
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f in fs:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0;}")
    prog.write_text("\n".join(lines))
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(prog), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = dict(l.rsplit(" ", 1) for l in out if l)
    for s in fields:
        cls = getattr(N, s)
        assert int(got[s]) == ctypes.sizeof(cls), s
        for f in fields[s]:
            assert int(got[f"{s}.{f}"]) == getattr(cls, f).offset, f"{s}.{f}"


def test_no_cpu_fallback_without_library(monkeypatch):
    from psgla_for_posterior_sampling_amd import _native as N
    monkeypatch.setattr(N, "_lib", None)
    monkeypatch.setattr(N, "LIB_PATH", "/nonexistent/libpsgla_hip.so")
    with pytest.raises(N.NativeLibraryError):
        N.lib()


def test_kernel_dispatch_rules_on_the_host():
    """psgla_tv_step_kernel is a host-side query (launches nothing; without a GPU the CU count defaults to the
    MI355X's 256): the fused-step kernel choice for the bench shape, the strong-scaling split, the reference's
    image shapes at the CLI's batch sizes, forced variants and the rejected ones."""
    from psgla_for_posterior_sampling_amd import _native as N
    lib = N.lib()
    BAND, STREAM, TILE = 0, 1, 3

    def kind(B, H, W, ldw=0, n_tv=10, variant=0, alpha1=True, exact=False):
        d = N.PsglaTvStep()
        d.B, d.C, d.H, d.W, d.ldw, d.n_tv, d.kernel_variant, d.exact = B, 3, H, W, ldw, n_tv, variant, int(exact)
        if not alpha1:
            d.x2[0], d.x2[1] = 16, 32          # non-null: alpha != 1 (the query never dereferences them)
        k = lib.psgla_tv_step_kernel(ctypes.byref(d))
        return k, (lib.psgla_last_error().decode() if k < 0 else "")

    assert kind(64, 256, 256)[0] == STREAM                       # BASELINE configs[1], one GPU
    assert kind(8, 256, 256)[0] == TILE                          # 8-GPU strong split: 240 tiles
    # round 6: no 72-row tiles, 48-row tiles at alpha = 1 only (the other instances spilled VGPRs)
    assert kind(12, 256, 256)[0] == TILE                         # 48-row tiles in two rounds
    assert kind(16, 256, 256)[0] == TILE                         # 4-GPU strong split: 480 tiles
    assert kind(20, 256, 256)[0] == STREAM                       # 600 tiles: three rounds
    assert kind(16, 256, 256, exact=True, variant=4)[0] == TILE  # forced: 48-row tiles in two rounds
    assert kind(8, 256, 256, exact=True)[0] == TILE              # 48-row tiles in one round: both modes
    assert kind(8, 256, 256, alpha1=False)[0] == STREAM          # alpha != 1: 32-row tiles would need 528
    assert kind(1, 256, 256, alpha1=False)[0] == TILE            # ... and fit for one image (32-row tiles)
    assert kind(64, 256, 256, alpha1=False)[0] == STREAM
    assert kind(1, 481, 321, ldw=324)[0] == TILE                 # castle at the CLI's batch 1
    assert kind(4, 481, 321, ldw=324)[0] == TILE                 # segmented rows: two rounds of tiles
    assert kind(8, 481, 321, ldw=324)[0] == STREAM
    assert kind(2, 321, 481, ldw=484)[0] == TILE
    assert kind(1, 256, 256, n_tv=14)[0] == TILE                 # n_tv > 10: no stream kernel
    assert kind(64, 256, 256, n_tv=14)[0] == BAND
    assert kind(64, 256, 256, variant=4)[0] == TILE              # forced variants
    assert kind(64, 256, 256, variant=1)[0] == BAND
    assert kind(8, 256, 256, variant=2)[0] == STREAM
    k, err = kind(64, 256, 256, variant=3)                       # the row-pair pipeline is gone (ABI 7)
    assert k == -1 and "kernel_variant" in err
    k, err = kind(1, 481, 321, ldw=324, variant=1)               # the band kernel needs ldw == W
    assert k == -1 and "row pitch" in err


def test_ctypes_arity_matches_header():
    """Every entry point's parameter count in include/psgla_hip.h equals the ctypes binding's (an ABI change that
    adds a parameter -- ABI 10's image width W of the noise entry points -- must reach both)."""
    from psgla_for_posterior_sampling_amd import _native as N
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    for name, (_res, args) in N._SIGNATURES.items():
        m = re.search(r"\b" + re.escape(name) + r"\s*\(([^)]*)\)\s*;", src)
        assert m, name
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(args), f"{name}: header {len(params)} vs ctypes {len(args)}"


def test_no_shipped_kernel_spills_vgprs():
    """Round 6 root cause of the rare tile-kernel faults / miscompares: a VGPR spilled to
    scratch inside a divergent (exec-masked) region is stored only for the active lanes and reloaded later for all
    of them, so the inactive lanes get stale values -- which then fed addresses on the early-stop redo path.  No kernel
    of the library may spill a VGPR (the code objects' own metadata, read from the shipped .so)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import code_object_meta
    from psgla_for_posterior_sampling_amd import _native as N
    ks = code_object_meta.kernels(N.LIB_PATH)
    assert len(ks) > 40, "no gfx950 code objects found in the library"
    spilled = {k[".name"]: k[".vgpr_spill_count"] for k in ks if k.get(".vgpr_spill_count", 0) > 0}
    assert not spilled, spilled
