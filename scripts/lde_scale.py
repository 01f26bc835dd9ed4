"""configs[4]-shape trace LDE launch sets (2^20 x 16, 7 columns per proof) for 1, 2 and 4 proofs in one
process: HIP-event ms per launch set and per proof (run under rocprofv3 --kernel-trace for per-kernel
durations). usage: python3 scripts/lde_scale.py [counts...]"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
import xfgstark  # noqa: E402
pr = xfgstark.XfgBurnMintProver()
for k in [int(x) for x in sys.argv[1:]] or [1, 2, 4]:
    ms = pr.bench_lde(k, 1 << 20, 16, int(os.environ.get("ITERS", "8")))
    print(f"proofs {k}: {ms:.3f} ms per launch set, {ms / k:.3f} ms per proof", flush=True)
