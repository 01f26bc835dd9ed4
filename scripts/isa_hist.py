"""Static VALU histogram of the gfx950 kernels of one source file (host-side, no GPU): compiles the
device code to assembly and prints per kernel the VALU instruction count, waterfall-loop markers
(v_readfirstlane / s_and_saveexec: a buffer descriptor or scalar operand the compiler could not
prove uniform) and the global-memory instruction forms.
usage: python3 scripts/isa_hist.py xfg-stark_amd/csrc/kernels.hip [kernel-substring] [--ops]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
show_ops = "--ops" in sys.argv
with tempfile.TemporaryDirectory() as d:
    out = os.path.join(d, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-o", out, os.path.abspath(src)], check=True, cwd=d, stderr=subprocess.DEVNULL)
    s = open(out).read()
for k in re.findall(r"^(_ZN3xfg\w+):", s, re.M):
    if pat not in k:
        continue
    i = s.index(k + ":")
    body = s[i:s.index("s_endpgm", i)]
    c = collections.Counter(l.strip().split()[0] for l in body.splitlines()
                            if l.strip() and not l.strip().startswith((".", ";", "_")) and not l.strip().endswith(":"))
    v = sum(n for o, n in c.items() if o.startswith("v_"))
    mem = {o: n for o, n in c.items() if o.startswith(("global_", "buffer_"))}
    print(f"{k[:64]:64s} valu={v:6d} readfirstlane={c['v_readfirstlane_b32']:3d} "
          f"saveexec={c['s_and_saveexec_b64']:3d} {mem}")
    if show_ops:
        for o, n in sorted(c.items(), key=lambda x: -x[1]):
            if o.startswith(("v_", "ds_")):
                print(f"    {o:28s}{n}")
