"""VALU issue ceiling of an instruction mix (round 5): the measured issue rate of each instruction
form (scripts/ubench/valu_ubench.hip, profiles/r05/valu_ubench.txt) applied to a kernel's static
instruction mix (hipcc --cuda-device-only -S listing), harmonic by count -- the lane-instructions/s
the VALU sustains on that mix at full occupancy. With a ledger (valu_per_proof.json) the per-kernel
ceilings combine, weighted by each kernel's share of a proof's lane instructions, into the whole-proof
ceiling, written back into the ledger (bench.py's whole_proof.valu reads it).
usage: valu_ceiling.py LISTING.s [LISTING2.s ...] --ledger profiles/r05/valu_per_proof.json"""
import collections
import json
import re
import sys

# T lane-ops/s (profiles/r05/valu_ubench.txt)
E64_SIMPLE = {"v_add_u32_e64", "v_sub_u32_e64", "v_subrev_u32_e64", "v_xor_b32_e64", "v_and_b32_e64",
              "v_or_b32_e64", "v_lshrrev_b32_e64", "v_lshlrev_b32_e64"}
E32_SIMPLE = {"v_add_u32_e32", "v_sub_u32_e32", "v_subrev_u32_e32", "v_xor_b32_e32", "v_and_b32_e32",
              "v_or_b32_e32", "v_lshrrev_b32_e32", "v_lshlrev_b32_e32", "v_mov_b32_e32", "v_not_b32_e32"}
RATE_E64, RATE_E32, RATE_BITOP3_CONST, RATE_OTHER = 66.0, 47.5, 66.0, 36.0


def rate(op, line):
    if op in E64_SIMPLE:
        return RATE_E64
    if op in E32_SIMPLE:
        return RATE_E32
    if op == "v_bitop3_b32":
        srcs = line.split(",")[1:4]
        return RATE_BITOP3_CONST if any(re.fullmatch(r"\s*-?(0x[0-9a-f]+|\d+)\s*", x) for x in srcs) else RATE_OTHER
    return RATE_OTHER


def kernels(paths):
    out, cur = {}, None
    for path in paths:
        for line in open(path):
            m = re.match(r"^(_Z\S*):", line)
            if m:
                cur = out.setdefault(m.group(1), [])
                continue
            if line.startswith(".Lfunc_end"):
                cur = None
            s = line.strip()
            if cur is not None and s.startswith("v_"):
                cur.append((s.split()[0], s))
    return out


def ceiling(instrs):
    if not instrs:
        return None
    return len(instrs) / sum(1.0 / rate(op, ln) for op, ln in instrs)


def demangled_match(ledger_name, mangled):
    # "void xfg::leaves_lde_kernel<7, 3>" -> name + template args as they appear mangled
    m = re.search(r"xfg::(\w+)(<([^>]*)>)?", ledger_name)
    if not m:
        return False
    name, args = m.group(1), m.group(3)
    if f"{len(name)}{name}" not in mangled:
        return False
    if args is None:
        return "ILi" not in mangled.split(f"{len(name)}{name}")[1][:4]
    want = "I" + "".join("Lb1E" if a.strip() == "true" else "Lb0E" if a.strip() == "false" else f"Li{a.strip()}E"
                         for a in args.split(",")) + "E"
    return (f"{len(name)}{name}" + want) in mangled


def main():
    args = sys.argv[1:]
    ledger = None
    if "--ledger" in args:
        i = args.index("--ledger")
        ledger = args[i + 1]
        args = args[:i] + args[i + 2:]
    ks = kernels(args)
    if not ledger:
        for k, v in sorted(ks.items(), key=lambda x: -len(x[1]))[:20]:
            print(f"{ceiling(v) or 0:6.1f} T  {len(v):6d} VALU  {k[:90]}")
        return
    d = json.load(open(ledger))
    tot, t_sum, per = 0.0, 0.0, {}
    for name, lanes in d["by_kernel"].items():
        cands = [v for k, v in ks.items() if demangled_match(name, k)]
        c = ceiling(cands[0]) if cands else None
        c = c or RATE_OTHER
        per[name] = round(c, 1)
        tot += lanes
        t_sum += lanes / c
    d["ceiling_T_lane_instr_s"] = round(tot / t_sum, 1)
    d["ceiling_by_kernel"] = {k: per[k] for k in list(d["by_kernel"])[:12]}
    d["ceiling_method"] = ("per-kernel harmonic issue rate of the static instruction mix (scripts/valu_ceiling.py: "
                           "two-source e64 simple ops 66, their e32 forms 47.5, bitop3 with a constant 66, every other "
                           "VALU form 36 T lane-ops/s, profiles/r05/valu_ubench.txt), weighted by the kernels' "
                           "lane instructions per proof")
    json.dump(d, open(ledger, "w"), indent=1)
    print(d["ceiling_T_lane_instr_s"], d["ceiling_by_kernel"])


if __name__ == "__main__":
    main()
