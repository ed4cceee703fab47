# Variant: all_clamp.py plus every fast iteration constant (tau, rho, sigma) of the stream, tile and band kernels as a
# VGPR operand (3-read fmas: the VGPR-bank lottery instead of the SGPR price).
import os
import runpy

_b = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "all_clamp.py"))
PATCHES = list(_b["PATCHES"]) + [
    ("xv = __builtin_fmaf(a.tau, yv[r][k] - tt, xo) * vconst(a.inv_opt);",
     "xv = __builtin_fmaf(vconst(a.tau), yv[r][k] - tt, xo) * vconst(a.inv_opt);", 1),
    ("xv = __builtin_fmaf(a.tau, yy[kk] - tt, xo) * vconst(a.inv_opt);",
     "xv = __builtin_fmaf(vconst(a.tau), yy[kk] - tt, xo) * vconst(a.inv_opt);", 1),
    ("xn = __builtin_fmaf(a.rho, xv - xo, xo);", "xn = __builtin_fmaf(vconst(a.rho), xv - xo, xo);", 3),
    ("const float sg0 = down ? a.sig_tv : 0.f;", "const float sg0 = down ? vconst(a.sig_tv) : 0.f;", 1),
    ("const float v0 = __builtin_fmaf(a.sig_tv, g0, uo0);", "const float v0 = __builtin_fmaf(vconst(a.sig_tv), g0, uo0);", 2),
    ("const float v1 = __builtin_fmaf(a.sig_tv, g1, uo1);", "const float v1 = __builtin_fmaf(vconst(a.sig_tv), g1, uo1);", 2),
    ("__builtin_fmaf(a.rho, __builtin_fmaf(v0, f, -uo0), uo0);", "__builtin_fmaf(vconst(a.rho), __builtin_fmaf(v0, f, -uo0), uo0);", 3),
    ("__builtin_fmaf(a.rho, __builtin_fmaf(v1, f, -uo1), uo1);", "__builtin_fmaf(vconst(a.rho), __builtin_fmaf(v1, f, -uo1), uo1);", 3),
]
