# r03 u2 stores of the tile kernel (each dwordx4 instruction writes every other 16 B of a 2 KB span, sc1)
PATCHES = [(
    "            if (lo ? corelane : corelane_o) st_tile(lo ? pa : pb, lo ? A : B4);\n"
    "            if (lo ? corelane_o : corelane) st_tile(lo ? pb : pa, lo ? B4 : A);\n",
    "            if (corelane) { st_tile(pa, A); st_tile(pa + 4, make_float4(Bv[0], Bv[1], Bv[2], Bv[3])); }\n",
    1)]
