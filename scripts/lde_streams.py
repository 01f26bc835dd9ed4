"""Experiment (round 6): the trace-LDE launch set split over S streams, so that pass A of one chunk can
run beside pass B of another (pass A is VALU-bound, pass B near the copy rate). Needs a library built
with -DXFG_EXP_LDE_STREAMS (the xfg_bench_lde branch of commit "experiment: multi-stream LDE launch set",
removed from the product after it measured no gain: profiles/r06/lde_streams.txt). Run with XFG_LIB
pointing at that build."""
import os, sys
ROOT = "/root/repo" if os.path.exists("/root/repo/xfg-stark_amd") else "."
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
import xfgstark
pr = xfgstark.XfgBurnMintProver()
for rep in range(2):
    for S in ["0", "1", "2", "4", "8"]:
        if S == "0":
            os.environ.pop("XFG_EXP_S", None)
        else:
            os.environ["XFG_EXP_S"] = S
        ms = pr.bench_lde(64, 1 << 16, 8, 110)
        ms5 = pr.bench_lde(4, 1 << 20, 16, 36)
        print(f"S={S}: 2^16x8 64 proofs {ms:.3f} ms ({2113929216/ms/1e9*1e3/8000:.3f} of HBM)   2^20x16 4 proofs {ms5:.3f} ms", flush=True)
