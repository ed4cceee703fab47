"""Timing variant (bit-identical results): the row stream's stage waves at issue priority 2 (product: 1)."""
PATCHES = [("        __builtin_amdgcn_s_setprio(1);\n", "        __builtin_amdgcn_s_setprio(2);\n", 1)]
