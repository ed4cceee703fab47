"""Timing variant: the row stream's front waves at issue priority 1 (the product: 0; stages 1, back 3)."""
PATCHES = [("        // ---------------- FRONT state ----------------\n",
            "        // ---------------- FRONT state ----------------\n        __builtin_amdgcn_s_setprio(1);\n", 1)]
