# Diagnostic (wrong early stop): the tile kernel's rel-err partial sums written by plain stores instead of
# contended fp64 atomics -- what the atomics cost at the end of a tile
PATCHES = [
    ("""            atomicAdd(&nrm[((size_t)b * a.n_tv + t) * 2], sd);
            atomicAdd(&nrm[((size_t)b * a.n_tv + t) * 2 + 1], sn);""",
     """            nrm[((size_t)b * a.n_tv + t) * 2] = sd;
            nrm[((size_t)b * a.n_tv + t) * 2 + 1] = sn;""", 1),
]
