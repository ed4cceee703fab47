"""Timing-only variant (wrong samples): the stream kernel's front computes no noise (no Philox, no Box-Muller;
Z = 0) -- what the noise costs the 64-chain step."""
PATCHES = [
    ("philox4x32_10(c0, c1, c2, c3, (uint32_t)a.seed, (uint32_t)(a.chain0 + g.bb));", "", 1),
    ("box_muller(ph0, ph1, zn0, zn1);", "zn0 = zn1 = 0.f;", 1),
    ("box_muller(ph2, ph3, zn2, zn3);", "zn2 = zn3 = 0.f;", 1),
]
