"""The tile kernel with the rel-err sums before the u2 stores for every tile shape (before round 4's late sums)."""
PATCHES = [("    constexpr bool RELERR_LATE = NW == 16;", "    constexpr bool RELERR_LATE = false;", 1)]
