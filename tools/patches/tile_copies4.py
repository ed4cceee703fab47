# Variant: norm copies for few-tile chains too (8 chains of 30 tiles: 4 copies, read by the spread finaliser).
PATCHES = [("            if (s.norm_copies < 1 || s.C * s.nbands * s.st_nsegs < 64) s.norm_copies = 1;",
            "            if (s.norm_copies < 1) s.norm_copies = 1;\n"
            "            if (s.C * s.nbands * s.st_nsegs < 64) s.norm_copies = s.B * 8 <= 32 ? min(s.norm_copies, 8) : (s.B * 4 <= 32 ? min(s.norm_copies, 4) : 1);", 1)]
