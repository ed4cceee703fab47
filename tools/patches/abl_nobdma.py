"""Timing-only ablation (wrong data): the row stream's back issues no LDS-DMA loads (previous mean / sq)."""
PATCHES = [
    ("        auto back_issue = [&](int q, const RowCursor& rc) {\n",
     "        auto back_issue = [&](int q, const RowCursor& rc) {\n            if (q >= 0) return;\n", 1),
]
