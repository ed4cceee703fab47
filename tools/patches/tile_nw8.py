# A/B: the 32- and 48-row tiles as 8 waves x 4 / 6 rows instead of 16 waves x 2 / 3 rows (same geometry)
PATCHES = [
    ("            a.tile_r = 3;\n            a.tile_nw = 16;", "            a.tile_r = 6;\n            a.tile_nw = 8;", 1),
    ("                a.tile_r = 2;\n                a.tile_nw = 16;", "                a.tile_r = 4;\n                a.tile_nw = 8;", 1),
]
