"""The generated BLAKE3 half-round blocks (xfg-stark_amd/csrc/b3_sched.inc, scripts/b3_sched_gen.py)
checked on the CPU: every asm block, interpreted instruction by instruction, computes the four G
functions of a BLAKE3 half-round (the round function of the BLAKE3 spec, section 2.2) for random
states and messages with the block's zero words; the committed header is what the generator emits;
and the half-round blocks chained into seven rounds reproduce the BLAKE3 compression of the
oracle's BLAKE3 (pinned to the published vectors, tests/test_oracle_kats.py) on element hashes."""
import os
import random
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "xfg-stark_amd", "csrc", "b3_sched.inc")
GEN = os.path.join(ROOT, "scripts", "b3_sched_gen.py")
M32 = 0xFFFFFFFF


def blocks():
    """{Z: [instruction lines]} from the header (Z = None: the generic block)"""
    text = open(INC).read()
    out = {}
    for m in re.finditer(r"(?:if constexpr \(Z == 0x([0-9a-f]+)u\)|else)\s*\n\s*asm\((.*?)\n\s*:", text, re.S):
        z = int(m.group(1), 16) if m.group(1) else None
        out[z] = [s.replace("\\n", "").strip() for s in re.findall(r'"([^"]*)"', m.group(2))]
    return out


def run_block(lines, ops):
    """interpret the block's instructions on operand values ops[0..23] (32-bit)"""
    v = list(ops)

    def r(tok):
        return int(tok.strip().lstrip("%"))

    for ln in lines:
        if ln.startswith("s_nop"):
            continue
        op, args = ln.split(None, 1)
        a = [t.strip() for t in args.split(",")]
        if op == "v_add3_u32":
            v[r(a[0])] = (v[r(a[1])] + v[r(a[2])] + v[r(a[3])]) & M32
        elif op == "v_add_u32_e64":
            v[r(a[0])] = (v[r(a[1])] + v[r(a[2])]) & M32
        elif op == "v_xor_b32_e64":
            v[r(a[0])] = v[r(a[1])] ^ v[r(a[2])]
        elif op == "v_alignbit_b32":
            x, n = v[r(a[1])], int(a[3])
            assert r(a[1]) == r(a[2])
            v[r(a[0])] = ((x >> n) | (x << (32 - n))) & M32
        else:
            raise AssertionError(f"unexpected instruction {ln}")
        assert r(a[0]) < 16, "a block writes only state operands"
    return v


def rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def g_ref(s, a, b, c, d, x, y):
    s[a] = (s[a] + s[b] + x) & M32
    s[d] = rotr(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & M32
    s[b] = rotr(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b] + y) & M32
    s[d] = rotr(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & M32
    s[b] = rotr(s[b] ^ s[c], 7)


def test_header_is_generated():
    want = subprocess.run([sys.executable, GEN, "--product", "/dev/stdout"], capture_output=True, text=True,
                          check=True).stdout
    assert open(INC).read() == want, "csrc/b3_sched.inc differs from scripts/b3_sched_gen.py --product"


def test_every_block_is_four_g_functions():
    bl = blocks()
    assert None in bl and len(bl) > 8
    rng = random.Random(5)
    for z, lines in bl.items():
        zz = z or 0
        valu = [ln for ln in lines if not ln.startswith("s_nop")]
        assert len(valu) == 48
        # a zero word's add3 is a two-source add, every other add3 stays
        assert sum(ln.startswith("v_add3_u32") for ln in valu) == 8 - bin(zz).count("1")
        for _ in range(20):
            st = [rng.getrandbits(32) for _ in range(16)]
            msg = [0 if zz >> j & 1 else rng.getrandbits(32) for j in range(8)]
            got = run_block(lines, st + msg)
            ref = list(st)
            for g in range(4):
                g_ref(ref, 4 * g, 4 * g + 1, 4 * g + 2, 4 * g + 3, msg[2 * g], msg[2 * g + 1])
            assert got[:16] == ref, f"block Z={z}"
            assert got[16:] == msg


def test_every_reached_mask_has_its_block():
    """every zero mask a device compression reaches (round 1's diagonal half and rounds 2..7 of each
    entry pattern of the element hashes) has its own block, so no half-round silently falls back to
    the generic Z = 0 block (the fallback is correct, only slower)"""
    sys.path.insert(0, os.path.dirname(GEN))
    import b3_sched_gen as G
    have = set(blocks()) - {None}
    for zm in G.ZERO_PATTERNS:
        z, reached = zm, [zm >> 8]
        for _ in range(6):
            z = G.perm_mask(z)
            reached += [z & 0xFF, z >> 8]
        for r in reached:
            assert r == 0 or r in have, f"entry mask {zm:#06x} reaches Z = {r:#04x} with no block"


PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
COL = [(0, 4, 8, 12), (1, 5, 9, 13), (2, 6, 10, 14), (3, 7, 11, 15)]
DIAG = [(0, 5, 10, 15), (1, 6, 11, 12), (2, 7, 8, 13), (3, 4, 9, 14)]


def compress_blocks(m, block_len, flags, zm):
    """BLAKE3 compression of one chunk-start block with the product's structure: round 1's column
    half as plain G functions, every other half-round through the generated block of its zero mask"""
    bl = blocks()
    s = IV + IV[:4] + [0, 0, block_len, flags]
    m = list(m)
    z = zm

    def half(quads, words, zmask):
        lines = bl.get(zmask, bl[None])
        ops = [s[i] for q in quads for i in q] + words
        out = run_block(lines, ops)
        k = 0
        for q in quads:
            for i in q:
                s[i] = out[k]
                k += 1

    for rnd in range(7):
        if rnd == 0:
            for g, q in enumerate(COL):
                g_ref(s, *q, m[2 * g], m[2 * g + 1])
        else:
            half(COL, m[:8], z & 0xFF)
        half(DIAG, m[8:], z >> 8)
        m = [m[PERM[i]] for i in range(16)]
        z = sum(((z >> PERM[i]) & 1) << i for i in range(16))
    return [s[i] ^ s[i + 8] for i in range(8)]


@pytest.mark.parametrize("k", [1, 2, 7, 8])
def test_chained_blocks_match_oracle_hash(k):
    """hash_elements of k field elements (one block) through the generated blocks == the oracle"""
    from oracle_lib import blake3  # the CPU restatement (test infrastructure)

    rng = random.Random(k)
    p = (1 << 64) - (1 << 32) + 1
    elems = [rng.randrange(p) for _ in range(k)]
    words = []
    for e in elems:
        words += [e & M32, e >> 32]
    words += [0] * (16 - len(words))
    zm = 0xFFFF & ~((1 << (2 * k)) - 1)
    out = compress_blocks(words, 8 * k, 1 | 2 | 8, zm)  # CHUNK_START | CHUNK_END | ROOT
    got = b"".join(w.to_bytes(4, "little") for w in out)
    assert got == blake3(b"".join(e.to_bytes(8, "little") for e in elems))
