# Variant (row stream only: in the 48-row tile the same made the allocator spill): the front's data-term multiply (inv_sigma2) and the back's accumulator coefficients (ca, cb) as VGPR
# operands (vconst): 2-source multiplies, so 2.17 instead of 4.24 SIMD cycles per wave-instruction with no bank risk.
PATCHES = [
    ("                        const float g = (mk[k] * (yo[k] - X[k])) * a.inv_sigma2;",
     "                        const float g = (mk[k] * (yo[k] - X[k])) * vconst(a.inv_sigma2);", 1),
    ("                            m[kk] = si.cb * xs[kk];\n                            qq[kk] = si.cb * (xs[kk] * xs[kk]);",
     "                            m[kk] = vconst(si.cb) * xs[kk];\n                            qq[kk] = vconst(si.cb) * (xs[kk] * xs[kk]);", 1),
    ("                            m[kk] = si.ca * ms[kk] + si.cb * xs[kk];\n                            qq[kk] = si.ca * qs[kk] + si.cb * (xs[kk] * xs[kk]);",
     "                            m[kk] = vconst(si.ca) * ms[kk] + vconst(si.cb) * xs[kk];\n                            qq[kk] = vconst(si.ca) * qs[kk] + vconst(si.cb) * (xs[kk] * xs[kk]);", 1),
]
