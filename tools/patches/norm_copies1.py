# A/B baseline: the tile kernel's rel-err sums on one copy of norms (ABI 8 descriptor's norms_copies ignored)
PATCHES = [
    ("    a.norm_copies = d->norms_copies > 1 ? d->norms_copies : 1;", "    a.norm_copies = 1;", 1),
]
