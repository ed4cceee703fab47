# Diagnostic (timing-only sensitivity, never in the product): 4 extra VALU issue slots per element in the tile
# kernel's primal (v_nop: an issue slot each, no registers -- fmas with a run-time zero spilled a VGPR).  Measures
# whether the iteration time follows VALU issue.
PATCHES = [(
    "                    xn = __builtin_fmaf(a.rho, xv - xo, xo);\n                }\n                // rel-err terms of the counted rows",
    "                    xn = __builtin_fmaf(a.rho, xv - xo, xo);\n"
    "                    asm volatile(\"v_nop\\n v_nop\\n v_nop\\n v_nop\");\n"
    "                }\n                // rel-err terms of the counted rows", 1)]
