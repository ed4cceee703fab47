# Diagnostic (timing-only sensitivity, never in the product): 4 extra VALU per element in the tile kernel's dual
# (v_nop).  See tile_valu_p4.py.
PATCHES = [(
    "                    u1[r][k] = __builtin_fmaf(a.rho, __builtin_fmaf(v1, f, -uo1), uo1);\n                }\n            }\n        }\n        }\n        if (act_d)",
    "                    u1[r][k] = __builtin_fmaf(a.rho, __builtin_fmaf(v1, f, -uo1), uo1);\n"
    "                    asm volatile(\"v_nop\\n v_nop\\n v_nop\\n v_nop\");\n"
    "                }\n            }\n        }\n        }\n        if (act_d)", 1)]
