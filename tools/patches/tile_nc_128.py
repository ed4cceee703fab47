"""Eight norm copies only from 128 tiles per chain (the rule before round 4's back-to-back copy reads)."""
PATCHES = [("if (s.norm_copies < 1 || s.C * s.nbands * s.st_nsegs < 64) s.norm_copies = 1;",
            "if (s.norm_copies < 1 || s.C * s.nbands * s.st_nsegs < 128) s.norm_copies = 1;", 1)]
