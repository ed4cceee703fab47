# timing: the tile kernel with 2 rows per wave (32-row tiles) wherever the tile kernel is selected
PATCHES = [
    ("    if (nsegs < 1 || R != 3) return 0;", "    if (nsegs < 1 || R < 2 || R > 3) return 0;", 1),
    ("hipLaunchKernelGGL((tv_tile_kernel<EXACT, ALPHA1, 3, false>)", "hipLaunchKernelGGL((tv_tile_kernel<EXACT, ALPHA1, 2, false>)", 1),
    ("hipLaunchKernelGGL((tv_tile_kernel<EXACT, ALPHA1, 3, true>)", "hipLaunchKernelGGL((tv_tile_kernel<EXACT, ALPHA1, 2, true>)", 1),
    ("        const int wg = tile_geometry(P, d->H, tile_segs, d->n_tv, 3, &bh, &nb);", "        const int wg = tile_geometry(P, d->H, tile_segs, d->n_tv, 2, &bh, &nb);", 1),
    ("            a.tile_r = 3;", "            a.tile_r = 2;", 1),
]
