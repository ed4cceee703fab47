# Variant: in the fast stream, tile and band kernels, the TV projection min(1, ths * rsq(s2)) as a clamp modifier
# on the multiply (fminf(fmaxf(x, 0), 1): bit-identical for x >= 0 and +inf) and the 2-read multiplies by kernel
# constants (ths, inv_opt) with the constant in a VGPR (vconst).  tools/valu_probe2: an SGPR source costs 4.24
# SIMD cycles per wave-instruction at 4 waves per SIMD, a VGPR one 2.17; v_min 4.24.
VCONST = ("__device__ __forceinline__ float2 row_sum2(float a, float b) {",
          "__device__ __forceinline__ float vconst(float s) {\n    float v;\n    asm(\"v_mov_b32 %0, %1\" : \"=v\"(v) : \"s\"(s));\n    return v;\n}\n"
          "__device__ __forceinline__ float2 row_sum2(float a, float b) {", 1)
PATCHES = [
    VCONST,
    ("xv = __builtin_fmaf(a.tau, yv[r][k] - tt, xo) * a.inv_opt;",
     "xv = __builtin_fmaf(a.tau, yv[r][k] - tt, xo) * vconst(a.inv_opt);", 1),
    ("xv = __builtin_fmaf(a.tau, yy[kk] - tt, xo) * a.inv_opt;",
     "xv = __builtin_fmaf(a.tau, yy[kk] - tt, xo) * vconst(a.inv_opt);", 1),
    ("const float f = fminf(1.0f, a.ths * __builtin_amdgcn_rsqf(s2));",
     "const float f = fminf(fmaxf(vconst(a.ths) * __builtin_amdgcn_rsqf(s2), 0.0f), 1.0f);", 3),
]
