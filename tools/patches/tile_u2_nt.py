# r03 u2 layout of the tile kernel's stores, but nt (not write-through) instead of sc1
PATCHES = [(
    "            if (lo ? corelane : corelane_o) st_tile(lo ? pa : pb, lo ? A : B4);\n"
    "            if (lo ? corelane_o : corelane) st_tile(lo ? pb : pa, lo ? B4 : A);\n",
    "            if (corelane) { st_nt(pa, A); st_nt(pa + 4, make_float4(Bv[0], Bv[1], Bv[2], Bv[3])); }\n",
    1)]
