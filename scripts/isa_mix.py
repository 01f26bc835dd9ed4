"""Static instruction mix of one kernel in a gfx950 assembly listing (hipcc --cuda-device-only -S):
python3 scripts/isa_mix.py file.s SYMBOL_SUBSTRING -> VALU / SALU / LDS / VMEM / s_nop counts and the
top opcodes (straight-line kernels: the static count is the per-thread dynamic count)."""
import collections
import re
import sys


def kernel_lines(path, sub):
    out, on = [], False
    for line in open(path):
        if re.match(r"^_Z\S*:", line):
            on = sub in line.split(":")[0]
            continue
        if on:
            if line.startswith("\t.section") or line.startswith(".Lfunc_end"):
                break
            s = line.strip()
            if s and not s.startswith((";", ".", "//")) and not s.endswith(":"):
                out.append(s.split()[0])
    return out


def main():
    ops = kernel_lines(sys.argv[1], sys.argv[2])
    c = collections.Counter(ops)
    cls = collections.Counter()
    for op, k in c.items():
        if op.startswith("v_"):
            cls["valu"] += k
        elif op.startswith("s_nop"):
            cls["s_nop"] += k
        elif op.startswith("s_"):
            cls["salu"] += k
        elif op.startswith("ds_"):
            cls["lds"] += k
        elif op.startswith(("global_", "buffer_", "flat_")):
            cls["vmem"] += k
    print(dict(cls), "total", len(ops))
    for op, k in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
        print(f"{k:6d} {op}")


if __name__ == "__main__":
    main()
