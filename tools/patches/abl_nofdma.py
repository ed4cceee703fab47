"""Timing-only ablation (wrong data): the row stream's front issues no LDS-DMA loads (X, y, u2, mask)."""
PATCHES = [
    ("        auto front_issue = [&](int part, int q, const RowCursor& rc) {\n",
     "        auto front_issue = [&](int part, int q, const RowCursor& rc) {\n            if (part >= 0) return;\n", 1),
]
