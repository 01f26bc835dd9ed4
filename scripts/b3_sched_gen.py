#!/usr/bin/env python3
"""Generate BLAKE3 half-round schedules as single inline-asm strings for gfx950.

A half-round is four independent G functions (column or diagonal), 48 VALU: per G
add3 / xor / rot16 / add / xor / rot12 / add3 / xor / rot8 / add / xor / rot7.  Operands %0..%15
are the states (a0 b0 c0 d0 a1 b1 c1 d1 ...), %16..%23 the message words (x0 y0 x1 y1 ...).
Each schedule is an ORDER of the (G, step) pairs that respects every G's own step order, plus a
NOP policy (`s_nop 0` after chosen instructions -- on gfx950 a fast/slow VALU mix issues faster
with them, profiles/r05/valu_mix.txt).  `--header` writes the C string macros.
"""
import argparse

# (kind, dst, src) with state names a b c d, message x y; kind: 'add3' 'xor' 'rot' 'add'
STEPS = [("add3", "a", "b", "x"), ("xor", "d", "a"), ("rot", "d", 16), ("add", "c", "d"),
         ("xor", "b", "c"), ("rot", "b", 12), ("add3", "a", "b", "y"), ("xor", "d", "a"),
         ("rot", "d", 8), ("add", "c", "d"), ("xor", "b", "c"), ("rot", "b", 7)]
SLOW = {"add3", "rot"}


def reg(g, n):
    return "%" + str(4 * g + "abcd".index(n)) if n in "abcd" else "%" + str(16 + 2 * g + "xy".index(n))


def instr(g, k):
    s = STEPS[k]
    if s[0] == "add3":
        return f"v_add3_u32 {reg(g, s[1])}, {reg(g, s[1])}, {reg(g, s[2])}, {reg(g, s[3])}"
    if s[0] == "xor":
        return f"v_xor_b32_e64 {reg(g, s[1])}, {reg(g, s[1])}, {reg(g, s[2])}"
    if s[0] == "add":
        return f"v_add_u32_e64 {reg(g, s[1])}, {reg(g, s[1])}, {reg(g, s[2])}"
    return f"v_alignbit_b32 {reg(g, s[1])}, {reg(g, s[1])}, {reg(g, s[1])}, {s[2]}"


def order(name):
    """list of (g, k)"""
    if name == "gbyg":
        return [(g, k) for g in range(4) for k in range(12)]
    if name == "lock":
        return [(g, k) for k in range(12) for g in range(4)]
    if name == "pairs":  # (G0 k, G1 k, G0 k+1, G1 k+1, G2 k, G3 k, G2 k+1, G3 k+1)
        out = []
        for k in range(0, 12, 2):
            for h in (0, 2):
                out += [(h, k), (h + 1, k), (h, k + 1), (h + 1, k + 1)]
        return out
    if name == "lockxr":  # step k of all four, then (k+1, k+2) of each G
        out = []
        for k in range(0, 12, 3):
            out += [(g, k) for g in range(4)]
            for g in range(4):
                out += [(g, k + 1), (g, k + 2)]
        return out
    if name.startswith("stag"):  # G g lags G0 by g*lag steps; round-robin over G's each tick
        lag = int(name[4:])
        out, t = [], 0
        while len(out) < 48:
            for g in range(4):
                k = t - g * lag
                if 0 <= k < 12:
                    out.append((g, k))
            t += 1
        return out
    if name == "alt":  # greedy: alternate fast / slow, independent of the previous instruction
        done = [0] * 4
        out, last_slow, last_g = [], True, -1
        while len(out) < 48:
            cands = [g for g in range(4) if done[g] < 12]
            want_slow = not last_slow
            pick = None
            for pref in ([g for g in cands if (STEPS[done[g]][0] in SLOW) == want_slow and g != last_g],
                         [g for g in cands if g != last_g], cands):
                if pref:
                    pick = min(pref, key=lambda g: done[g])
                    break
            out.append((pick, done[pick]))
            last_slow = STEPS[done[pick]][0] in SLOW
            last_g = pick
            done[pick] += 1
        return out
    raise ValueError(name)


def schedule(oname, nop):
    seq = order(oname)
    assert sorted(seq) == sorted((g, k) for g in range(4) for k in range(12))
    for g in range(4):
        ks = [k for (h, k) in seq if h == g]
        assert ks == sorted(ks)
    lines = []
    for i, (g, k) in enumerate(seq):
        lines.append(instr(g, k))
        slow = STEPS[k][0] in SLOW
        nxt = seq[i + 1] if i + 1 < len(seq) else None
        nxt_slow = nxt is not None and STEPS[nxt[1]][0] in SLOW
        if nop == "slow" and slow or nop == "fast" and not slow or nop == "all":
            lines.append("s_nop 0")
        elif nop == "fast1" and not slow:
            lines.append("s_nop 1")
        elif nop == "fs" and not slow and nxt_slow or nop == "sf" and slow and nxt is not None and not nxt_slow:
            lines.append("s_nop 0")
        elif nop == "ff" and not slow and nxt is not None and not nxt_slow:
            lines.append("s_nop 0")
        elif nop == "dep" and nxt is not None and nxt[0] == g:
            lines.append("s_nop 0")
    return lines


VARIANTS = [(o, n) for o in ("gbyg", "lock", "pairs", "lockxr", "stag1", "stag2", "stag3", "alt")
            for n in ("none", "slow", "fast", "fast1", "fs", "sf", "ff", "dep", "all")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--header", help="write the string macros for VARIANTS (ubench) to this path")
    ap.add_argument("--print", nargs=2, metavar=("ORDER", "NOP"))
    ap.add_argument("--ubench", help="write the ubench kernels for VARIANTS to this path")
    ap.add_argument("--product", help="write the product's schedule header (PRODUCT list) to this path")
    a = ap.parse_args()
    if a.product:
        product_header(a.product)
    if a.ubench:
        ubench_source(a.ubench)
    if a.print:
        print("\n".join(schedule(*a.print)))
    if a.header:
        with open(a.header, "w") as f:
            f.write("// generated by scripts/b3_sched_gen.py -- BLAKE3 half-round schedules\n#pragma once\n")
            for i, (o, n) in enumerate(VARIANTS):
                body = "".join(f'"{l}\\n"' for l in schedule(o, n))
                f.write(f"#define B3H_{i} {body}\n")
            f.write(f"#define B3H_COUNT {len(VARIANTS)}\n")
            f.write("static const char* b3h_names[] = {" + ", ".join(f'"{o}/{n}"' for o, n in VARIANTS) + "};\n")


def ubench_source(path):
    """the compression ubench over every VARIANT (scripts/ubench/b3sched_ubench.hip includes it)"""
    with open(path, "w") as f:
        f.write("// generated by scripts/b3_sched_gen.py --ubench\n")
        for i, (o, n) in enumerate(VARIANTS):
            body = "".join(f'"{l}\\n"' for l in schedule(o, n))
            f.write(f"__global__ __launch_bounds__(256) void kb{i}(uint32_t* out, int iters) {{ KB_PROLOGUE\n"
                    f"  for (int it = 0; it < iters; it++) {{\n#pragma unroll\n  for (int r = 0; r < 7; r++) {{\n"
                    f"    asm volatile({body} : B3_COL_OPS);\n"
                    f"    asm volatile({body} : B3_DIAG_OPS);\n    B3_PERMUTE_M;\n  }}\n  KB_OUT_XOR }}\n  KB_EPILOGUE }}\n")
        f.write("struct KB { const char* n; void (*f)(uint32_t*, int); } kbs[] = {" +
                ", ".join(f'{{"{o}/{n}", kb{i}}}' for i, (o, n) in enumerate(VARIANTS)) + "};\n")


# the product's candidates: XFG_B3_SCHED selects one at compile time (0 is the default)
PRODUCT = [("alt", "fast"), ("gbyg", "slow"), ("gbyg", "fs"), ("alt", "fs"), ("pairs", "fast")]


def product_header(path):
    with open(path, "w") as f:
        f.write("// generated by scripts/b3_sched_gen.py --product: one BLAKE3 half-round (four G functions,\n"
                "// 48 VALU) as one asm string; operands %0..%15 = a0 b0 c0 d0 .. a3 b3 c3 d3, %16..%23 = x0 y0 ..\n"
                "// x3 y3. XFG_B3_SCHED picks the order / s_nop policy (profiles/r05/b3_sched.txt).\n#pragma once\n"
                "#ifndef XFG_B3_SCHED\n#define XFG_B3_SCHED 0\n#endif\n")
        for i, (o, n) in enumerate(PRODUCT):
            body = "".join(f'"{l}\\n" ' for l in schedule(o, n))
            f.write(f"{'#if' if i == 0 else '#elif'} XFG_B3_SCHED == {i}  // {o} / s_nop after {n}\n"
                    f"#define XFG_B3_HALF_ASM {body}\n")
        f.write("#endif\n")


if __name__ == "__main__":
    main()
