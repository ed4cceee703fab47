# Diagnostic (never in the product): tools/patches/tile_phasediag.py plus the shader clock over the inner iterations.
# Slot 7 of each workgroup's stamps holds s_memtime (shader-clock ticks) elapsed between stamps 2 and 3, so
# tools/tile_phasediag.py (TDIAG_CLOCK=1) prints the clock the iterations ran at: ticks / (real-time span).
import os
import runpy

_base = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tile_phasediag.py"))
PATCHES = []
for old, new, count in _base["PATCHES"]:
    if "tdiag(step, 2);" in new:
        new = new.replace("if (track) tdiag(step, 2);",
                          "if (track) tdiag(step, 2);\n    const unsigned long long mt2 = __builtin_amdgcn_s_memtime();")
    if "tdiag(step, 3);" in new:
        new = new.replace(
            "if (track) tdiag(step, 3);",
            "if (track) tdiag(step, 3);\n    if (track && g_tdiag && __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0)\n"
            "        g_tdiag[((size_t)(step & 1) * 4096 + blockIdx.x) * 8 + 7] = __builtin_amdgcn_s_memtime() - mt2;")
    PATCHES.append((old, new, count))
