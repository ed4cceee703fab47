"""Eight norm copies for every tile launch (the product keeps one copy below 128 tiles per chain)."""
PATCHES = [("if (s.norm_copies < 1 || s.C * s.nbands * s.st_nsegs < 128) s.norm_copies = 1;",
            "if (s.norm_copies < 1) s.norm_copies = 1;", 1)]
