# Diagnostic (never in the product): tools/patches/tile_phasediag.py plus the finaliser's count of tiles whose rel-err
# partials leave a stop possible (sh.s_nuncert) in slot 7 of the finalising workgroup (tools/tile_phasediag.py
# TDIAG_NUNC=1 prints it).
import os
import runpy

_base = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tile_phasediag.py"))
PATCHES = list(_base["PATCHES"]) + [
    ("    const bool nostop = sh.s_nuncert == 0;\n",
     "    const bool nostop = sh.s_nuncert == 0;\n"
     "    if (g_tdiag && threadIdx.x == 0) g_tdiag[((size_t)(step & 1) * 4096 + blockIdx.x) * 8 + 7] = (unsigned long long)sh.s_nuncert;\n", 1),
]
