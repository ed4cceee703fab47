# Variant: fb_vconst.py plus the front's c1 / c2 fmas with VGPR coefficients (3-source: the VGPR-bank lottery).
import os
import runpy

_b = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "fb_vconst.py"))
PATCHES = list(_b["PATCHES"]) + [
    ("                        Yv[k] = okf ? __builtin_fmaf(a.c2, Z[k], __builtin_fmaf(a.c1, g, X[k])) : 0.f;",
     "                        Yv[k] = okf ? __builtin_fmaf(vconst(a.c2), Z[k], __builtin_fmaf(vconst(a.c1), g, X[k])) : 0.f;", 1),
]
