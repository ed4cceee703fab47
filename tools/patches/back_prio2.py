"""Timing variant (bit-identical results): the row stream's back waves at issue priority 2 (product: 3)."""
PATCHES = [("        __builtin_amdgcn_s_setprio(3);\n", "        __builtin_amdgcn_s_setprio(2);\n", 1)]
