"""configs[4] pipelined throughput for several (proofs per call, calls in flight) settings, one process:
bench.config5's measurement with its batch / depth varied. usage: python3 scripts/c5_depth.py B:D ..."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "xfg-stark_amd"), ROOT]
import torch  # noqa: E402
torch.cuda.init()
import xfgstark  # noqa: E402
import bench  # noqa: E402
p = xfgstark.XfgBurnMintProver()
for spec in sys.argv[1:]:
    b, d = (int(x) for x in spec.split(":"))
    c5 = bench.config5(p, 0, batch=b, calls=max(8, 2 * d), depth=d)
    print(f"batch {b} depth {d}: {c5['proofs_per_s']} proofs/s, {c5['device_bytes_added'] / 1e9:.1f} GB", flush=True)
p.close()
