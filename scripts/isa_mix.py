"""static instruction mix of kernels in a gfx950 .s file: python3 isa_mix.py file.s pattern [top]"""
import collections, re, sys

src, pat = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
text = open(src).read()
for m in re.finditer(r"^(_Z\S+):", text, re.M):
    name = m.group(1)
    if not re.search(pat, name):
        continue
    body = text[m.end():text.find(".Lfunc_end", m.end())]
    c = collections.Counter()
    for line in body.split("\n"):
        line = line.strip()
        if not line or line[0] in ".;_" or line.endswith(":"):
            continue
        c[line.split()[0]] += 1
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    print(f"{name}: {valu} VALU, {sum(c.values())} total")
    for k, v in c.most_common(top):
        print(f"   {k:28s} {v}")
