"""Timing variant (bit-identical results): stages 1-5 at issue priority 1, stages 6-10 at 2 (the pipeline's later
half drains first)."""
PATCHES = [("        __builtin_amdgcn_s_setprio(1);\n", "        if (k_st > 5) __builtin_amdgcn_s_setprio(2); else __builtin_amdgcn_s_setprio(1);\n", 1)]
