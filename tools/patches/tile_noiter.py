# timing-only (wrong results): the tile kernel without its inner TV iterations
PATCHES = [("""    const int wr0 = e0 + w * R, wr1 = wr0 + R;
    for (int it = 0; it < n_it; ++it) {""", """    const int wr0 = e0 + w * R, wr1 = wr0 + R;
    for (int it = 0; it < 0 * n_it; ++it) {""", 1)]
