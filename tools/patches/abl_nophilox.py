"""Timing-only ablation (wrong samples): the row stream's front runs no Philox rounds (its counters feed Box-Muller as
they are); run with --tv-tol 0."""
PATCHES = [
    ("philox4x32_10(c0, c1, c2, c3, (uint32_t)a.seed, (uint32_t)(a.chain0 + g.bb));",
     "c0 = c0 * 2654435761u; c1 ^= c0; c2 ^= c0 >> 7; c3 ^= c0 << 9;", 1),
]
