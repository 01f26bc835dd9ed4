"""BASELINE configs[1] latency probe: one 2^16-step burn proof (blowup 8, reference options) through
xfg_prove_burn_mint, synchronous, `reps` calls after one warm call (as bench.py's single_proof).

Run alone it prints the call times; run as
    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o single -- python3 scripts/single_proof.py 10 DIR/calls.txt
it also writes each timed call's [start, end] in CLOCK_MONOTONIC ns (the trace's clock), and
    python3 scripts/single_proof.py --summary DIR
splits the kernel trace by call: per call the kernel sum, the span from the first kernel's start to
the last kernel's end, and the call's wall time."""
import csv
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
sys.path.insert(0, ROOT)


def run(reps, calls_path):
    import synthetic
    import xfgstark
    pr = xfgstark.XfgBurnMintProver()
    n = 1 << 16
    kw = synthetic.burn_inputs(0)
    pr.prepare(1, n)  # every lane's workspace and code objects, as bench.py does before its timing
    pr.prove_burn_mint(**kw, trace_length=n)  # warm
    spans = []
    for _ in range(reps):
        t0 = time.perf_counter()
        pr.prove_burn_mint(**kw, trace_length=n)
        spans.append((t0, time.perf_counter()))
    pr.close()
    ms = [(b - a) * 1e3 for a, b in spans]
    print(f"single proof ms: best {min(ms):.3f} median {sorted(ms)[len(ms) // 2]:.3f} of {reps}")
    if calls_path:
        os.makedirs(os.path.dirname(os.path.abspath(calls_path)), exist_ok=True)
        with open(calls_path, "w") as f:
            for a, b in spans:
                f.write(f"{int(a * 1e9)} {int(b * 1e9)}\n")


def summary(d):
    calls = [tuple(map(int, l.split())) for l in open(os.path.join(d, "calls.txt"))]
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
          for r in csv.DictReader(open(glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]))]
    rows = []
    for a, b in calls:
        ks = [e for e in ev if a <= e[0] <= b]
        ksum = sum(e - s for s, e, _ in ks) / 1e6
        span = (max(e for _, e, _ in ks) - min(s for s, _, _ in ks)) / 1e6
        rows.append(((b - a) / 1e6, span, ksum, len(ks)))
        print(f"call {(b - a) / 1e6:8.3f} ms: {len(ks):4d} kernels, first start -> last end {span:8.3f} ms, "
              f"kernel sum {ksum:8.3f} ms")
    best = min(rows)
    print(f"best call {best[0]:.3f} ms: kernel span {best[1]:.3f} ms ({100 * best[1] / best[0]:.1f} % of the call), "
          f"kernel sum {best[2]:.3f} ms, {best[3]} kernels")
    # per kernel name over the best call
    a, b = calls[rows.index(best)]
    agg = {}
    for s, e, nm in ev:
        if a <= s <= b:
            k = nm.split("(")[0][:60]
            c, t = agg.get(k, (0, 0))
            agg[k] = (c + 1, t + e - s)
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {k:60s} x{c:3d} {t / 1e3:9.1f} us")


if __name__ == "__main__":
    if sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run(int(sys.argv[1]), sys.argv[2] if len(sys.argv) > 2 else None)
