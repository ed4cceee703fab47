"""Timing-only ablation (wrong samples): the row stream's front runs Philox but no Box-Muller (z = u32 scaled to
[-1, 1)); run with --tv-tol 0."""
PATCHES = [
    ("box_muller(ph0, ph1, zn0, zn1);", "zn0 = (float)(int)ph0 * 4.6566e-10f; zn1 = (float)(int)ph1 * 4.6566e-10f;", 1),
    ("box_muller(ph2, ph3, zn2, zn3);", "zn2 = (float)(int)ph2 * 4.6566e-10f; zn3 = (float)(int)ph3 * 4.6566e-10f;", 1),
]
