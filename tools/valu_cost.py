#!/usr/bin/env python3
"""Static VALU issue-cost model of a gfx950 assembly region, from the operand-form costs measured by
tools/valu_probe2 (profiles/r06q_valu_probe.txt; SIMD cycles per wave-instruction at 4 waves per SIMD):

    VOP2 / VOP1, VGPR or inline-constant sources, no bank conflict     2.17
    VOP3 (e64 / fma), VGPR or inline-constant sources, no conflict     2.57
    any SGPR source (VOP2 or VOP3)                                     4.24 / 4.30
    three VGPR reads (VOP3 fma, VOP2 fmac: dst is read) with two in the same bank (VGPR index mod 4)   4.24 / 4.39
    v_min / v_max / v_med3 / v_min3 (any sources)                      4.24 / 4.39
    DPP                                                                4.3
    v_pk_* (two lanes' worth)                                          4.3
    v_rsq / v_rcp / v_sqrt / v_exp / v_log                             8.24

Usage: python3 tools/valu_cost.py FILE.s FIRST_LINE LAST_LINE   (1-based, inclusive; e.g. one iteration loop)
Prints the per-class counts and cycles, the total, and the cycles a SIMD needs for 4 waves of it."""
import re
import sys
from collections import Counter

TRANS = ("v_rsq", "v_rcp", "v_sqrt", "v_exp", "v_log", "v_sin", "v_cos")
MINMAX = ("v_min", "v_max", "v_med3")


def vregs(ops):
    out = []
    for o in ops:
        o = o.strip().lstrip("-").replace("|", "")
        m = re.fullmatch(r"v(\d+)", o)
        if m:
            out.append(int(m.group(1)))
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", o)
        if m:
            out.append(int(m.group(1)))
    return out


def classify(line):
    parts = line.split(None, 1)
    op = parts[0]
    rest = parts[1] if len(parts) > 1 else ""
    rest = rest.split(";")[0]
    ops = [o.strip() for o in rest.split(",")]
    dst, srcs = ops[0], ops[1:]
    # DPP / modifiers trail the last source after a space
    srcs = [s.split(" ")[0] for s in srcs]
    has_s = any(re.fullmatch(r"-?\|?s\d+\|?|-?s\[\d+:\d+\]|vcc|exec|-?\|?ttmp\d+\|?", s) for s in srcs)
    vr = vregs(srcs)
    if op.startswith("v_fmac") or op.startswith("v_mac"):
        vr = vr + vregs([dst])
    banks = [r % 4 for r in vr]
    conflict = len(banks) >= 3 and len(set(banks)) < len(banks)
    vop3 = ("_e64" in op) or not (op.endswith("_e32") or "_dpp" in op or op.startswith("v_mov_b32") or
                                  op.startswith("v_readfirstlane") or op.startswith("v_readlane"))
    if any(op.startswith(t) for t in TRANS):
        return "transcendental", 8.24
    if "_dpp" in op or "row_" in line or "wave_sh" in line or "quad_perm" in line:
        return "dpp", 4.3
    if op.startswith("v_pk_"):
        return "packed", 4.3
    if any(op.startswith(t) for t in MINMAX):
        return "min/max", 4.39 if vop3 else 4.24
    if has_s:
        return ("vop3 sgpr" if vop3 else "vop2 sgpr"), (4.30 if vop3 else 4.24)
    if conflict:
        return ("vop3 bank conflict" if vop3 else "vop2 3-read bank conflict"), (4.39 if vop3 else 4.24)
    return ("vop3" if vop3 else "vop2"), (2.57 if vop3 else 2.17)


def main():
    path, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    lines = open(path).read().splitlines()[a - 1:b]
    cnt, cyc = Counter(), Counter()
    for ln in lines:
        s = ln.strip()
        if not s.startswith("v_") or s.startswith("v_cmp") or s.startswith("v_readfirstlane"):
            continue
        k, c = classify(s)
        cnt[k] += 1
        cyc[k] += c
    tot = sum(cyc.values())
    for k in sorted(cnt, key=lambda k: -cyc[k]):
        print(f"  {k:28s} {cnt[k]:5d} instr  {cyc[k]:8.1f} cyc")
    n = sum(cnt.values())
    print(f"  total {n} VALU, {tot:.1f} SIMD cycles per wave ({tot / max(n, 1):.2f} per instruction); "
          f"4 waves: {4 * tot:.0f} cycles")


if __name__ == "__main__":
    main()
