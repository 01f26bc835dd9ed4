#!/usr/bin/env python3
"""Generate BLAKE3 half-round schedules as single inline-asm strings for gfx950.

A half-round is four independent G functions (column or diagonal), 48 VALU: per G
add3 / xor / rot16 / add / xor / rot12 / add3 / xor / rot8 / add / xor / rot7.  Operands %0..%15
are the states (a0 b0 c0 d0 a1 b1 c1 d1 ...), %16..%23 the message words (x0 y0 x1 y1 ...).
Each schedule is an ORDER of the (G, step) pairs that respects every G's own step order, plus a
NOP policy (`s_nop 0` after chosen instructions -- on gfx950 a fast/slow VALU mix issues faster
with them, profiles/r05/b3_sched.txt). A zero mask Z (bit j: message operand %(16 + j) is known to
be zero) turns that word's three-source add3 into a two-source e64 add, a fast instruction.

  --ubench PATH   the compression ubench kernels for VARIANTS (scripts/ubench/b3sched_ubench.hip)
  --product PATH  the product header xfg-stark_amd/csrc/b3_sched.inc: b3_half<Z> for every zero
                  mask the device hashes meet (ZERO_PATTERNS), in the PRODUCT schedule
  --print ORDER NOP [Z]
"""
import argparse

# (kind, dst, src) with state names a b c d, message x y; kind: 'add3' 'xor' 'rot' 'add'
STEPS = [("add3", "a", "b", "x"), ("xor", "d", "a"), ("rot", "d", 16), ("add", "c", "d"),
         ("xor", "b", "c"), ("rot", "b", 12), ("add3", "a", "b", "y"), ("xor", "d", "a"),
         ("rot", "d", 8), ("add", "c", "d"), ("xor", "b", "c"), ("rot", "b", 7)]
SLOW = {"add3", "rot"}


def reg(g, n):
    return "%" + str(4 * g + "abcd".index(n)) if n in "abcd" else "%" + str(16 + 2 * g + "xy".index(n))


def kind(g, k, z):
    s = STEPS[k]
    if s[0] == "add3" and z >> (2 * g + "xy".index(s[3])) & 1:
        return "add2"  # a + b + 0
    return s[0]


def slow(g, k, z):
    return kind(g, k, z) in SLOW


def instr(g, k, z):
    s, kd = STEPS[k], kind(g, k, z)
    if kd == "add3":
        return f"v_add3_u32 {reg(g, s[1])}, {reg(g, s[1])}, {reg(g, s[2])}, {reg(g, s[3])}"
    if kd in ("add", "add2"):
        return f"v_add_u32_e64 {reg(g, s[1])}, {reg(g, s[1])}, {reg(g, s[2])}"
    if kd == "xor":
        return f"v_xor_b32_e64 {reg(g, s[1])}, {reg(g, s[1])}, {reg(g, s[2])}"
    return f"v_alignbit_b32 {reg(g, s[1])}, {reg(g, s[1])}, {reg(g, s[1])}, {s[2]}"


def order(name, z=0):
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
            for pref in ([g for g in cands if slow(g, done[g], z) == want_slow and g != last_g],
                         [g for g in cands if g != last_g], cands):
                if pref:
                    pick = min(pref, key=lambda g: done[g])
                    break
            out.append((pick, done[pick]))
            last_slow = slow(pick, done[pick], z)
            last_g = pick
            done[pick] += 1
        return out
    raise ValueError(name)


def schedule(oname, nop, z=0):
    seq = order(oname, z)
    assert sorted(seq) == sorted((g, k) for g in range(4) for k in range(12))
    for g in range(4):
        ks = [k for (h, k) in seq if h == g]
        assert ks == sorted(ks)
    lines = []
    for i, (g, k) in enumerate(seq):
        lines.append(instr(g, k, z))
        sl = slow(g, k, z)
        nxt = seq[i + 1] if i + 1 < len(seq) else None
        nxt_slow = nxt is not None and slow(nxt[0], nxt[1], z)
        if nop == "slow" and sl or nop == "fast" and not sl or nop == "all":
            lines.append("s_nop 0")
        elif nop == "fast1" and not sl:
            lines.append("s_nop 1")
        elif nop == "fs" and not sl and nxt_slow or nop == "sf" and sl and nxt is not None and not nxt_slow:
            lines.append("s_nop 0")
        elif nop == "ff" and not sl and nxt is not None and not nxt_slow:
            lines.append("s_nop 0")
        elif nop == "dep" and nxt is not None and nxt[0] == g:
            lines.append("s_nop 0")
    return lines


VARIANTS = [(o, n) for o in ("gbyg", "lock", "pairs", "lockxr", "stag1", "stag2", "stag3", "alt")
            for n in ("none", "slow", "fast", "fast1", "fs", "sf", "ff", "dep", "all")]
if __import__("os").environ.get("B3_VARIANTS"):  # e.g. B3_VARIANTS="alt/fast alt/none" (a shorter ubench)
    VARIANTS = [tuple(v.split("/")) for v in __import__("os").environ["B3_VARIANTS"].split()]


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


# the product's schedule (the candidate orders measured equal in the bench, profiles/r05/b3_sched.txt)
PRODUCT = ("alt", "fast")
# BLAKE3 message permutation: round r + 1 reads m'[i] = m[PERM[i]]
PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
# zero message words at compression entry of the device's element hashes: hash_elems<K> of K < 8
# elements leaves words 2K..15 zero (K = 7 trace rows, 1 and 2 the base / extension composition
# and constraint columns), and 40-byte digest || u64 blocks leave 10..15 zero
ZERO_PATTERNS = [sum(1 << w for w in range(2 * k, 16)) for k in (1, 2, 3, 4, 5, 6, 7)] + [
    sum(1 << w for w in range(10, 16))]


def perm_mask(z):
    return sum(1 << i for i in range(16) if z >> PERM[i] & 1)


def round_masks(zm):
    """16-bit zero masks of the message as rounds 2..7 read it"""
    out, z = [], zm
    for _ in range(6):
        z = perm_mask(z)
        out.append(z)
    return out


def product_masks():
    """every 8-bit half-round zero mask the device compression reaches: round 1's diagonal half
    (message words 8..15 of the entry mask; round 1's column half stays in C) and both halves of
    rounds 2..7"""
    masks = {0}
    for zm in ZERO_PATTERNS:
        masks.add(zm >> 8)
        for z in round_masks(zm):
            masks.add(z & 0xFF)
            masks.add(z >> 8)
    return masks


def product_header(path):
    masks = product_masks()
    ops = ('"+v"(a0), "+v"(b0), "+v"(c0), "+v"(d0), "+v"(a1), "+v"(b1), "+v"(c1), "+v"(d1), "+v"(a2), '
           '"+v"(b2), "+v"(c2), "+v"(d2), "+v"(a3), "+v"(b3), "+v"(c3), "+v"(d3) : "v"(x0), "v"(y0), "v"(x1), '
           '"v"(y1), "v"(x2), "v"(y2), "v"(x3), "v"(y3)')
    with open(path, "w") as f:
        f.write(f"// generated by scripts/b3_sched_gen.py --product: one BLAKE3 half-round (four G functions, 48\n"
                f"// VALU) as one asm block in the {PRODUCT[0]} order with an s_nop after each {PRODUCT[1]} "
                f"instruction\n// (profiles/r05/b3_sched.txt). Z: message words known to be zero (bit j = the "
                f"j-th of x0 y0 .. x3 y3),\n// whose add3 becomes a two-source e64 add; masks outside this list "
                f"use the Z = 0 block.\n#pragma once\n\n")
        f.write("template <unsigned Z>\n__device__ __forceinline__ void b3_half(uint32_t& a0, uint32_t& b0, "
                "uint32_t& c0, uint32_t& d0, uint32_t& a1,\n    uint32_t& b1, uint32_t& c1, uint32_t& d1, "
                "uint32_t& a2, uint32_t& b2, uint32_t& c2, uint32_t& d2, uint32_t& a3, uint32_t& b3,\n"
                "    uint32_t& c3, uint32_t& d3, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t x2, "
                "uint32_t y2,\n    uint32_t x3, uint32_t y3) {\n")
        first = True
        for z in sorted(masks - {0}):
            body = " ".join(f'"{l}\\n"' for l in schedule(*PRODUCT, z))
            f.write(f"    {'if' if first else 'else if'} constexpr (Z == 0x{z:02x}u)\n        asm({body}\n"
                    f"            : {ops});\n")
            first = False
        body = " ".join(f'"{l}\\n"' for l in schedule(*PRODUCT, 0))
        f.write(f"    else\n        asm({body}\n            : {ops});\n}}\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--print", nargs="+", metavar="ORDER NOP [Z]")
    ap.add_argument("--ubench", help="write the ubench kernels for VARIANTS to this path")
    ap.add_argument("--product", help="write the product's schedule header to this path")
    a = ap.parse_args()
    if a.product:
        product_header(a.product)
    if a.ubench:
        ubench_source(a.ubench)
    if a.print:
        z = int(a.print[2], 0) if len(a.print) > 2 else 0
        print("\n".join(schedule(a.print[0], a.print[1], z)))


if __name__ == "__main__":
    main()
