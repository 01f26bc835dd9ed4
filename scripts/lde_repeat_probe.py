"""Determinism probe of the configs[4] transforms: the 2^20 x 16 LDE (xfg_debug_lde) of the same
random polynomials REPS times, and the 2^21-point interpolation (xfg_debug_interpolate, offset 7);
prints each result's SHA-256 and how many words differ from the first result.
usage: python3 scripts/lde_repeat_probe.py [REPS] [NPOLY]   (XFG_LIB selects the build)"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))


def main():
    import numpy as np
    import torch
    torch.cuda.init()
    import xfgstark
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    npoly = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    P = 0xFFFFFFFF00000001
    rng = np.random.default_rng(7)
    pr = xfgstark.XfgBurnMintProver()
    n = 1 << 20
    coef = (rng.integers(0, 2**63, size=(npoly, n), dtype=np.uint64) % np.uint64(P)).astype(np.uint64)
    first = None
    for r in range(reps):
        out = pr.debug_lde(coef, n, 16)
        h = hashlib.sha256(out.tobytes()).hexdigest()[:16]
        nd = 0 if first is None else int(np.count_nonzero(out != first))
        if first is None:
            first = out.copy()
        print(f"lde rep {r}: {h} differing words {nd}", flush=True)
        if nd:  # natural index i = t + 16 m of polynomial p; m = k1 + 1024 k2 (pass B row k1, output k2)
            for p_, i in list(zip(*np.nonzero(out != first)))[:40]:
                t, m = int(i) % 16, int(i) // 16
                print(f"   poly {p_} coset {t} m {m} (k1 {m % 1024}, k2 {m // 1024}) got {int(out[p_, i]):#x} want {int(first[p_, i]):#x}")
    del first
    ev = (rng.integers(0, 2**63, size=(2, 2 * n), dtype=np.uint64) % np.uint64(P)).astype(np.uint64)
    first = None
    for r in range(reps):
        out = pr.debug_interpolate(ev, 2 * n, True) if "debug_interpolate" in dir(pr) else None
        if out is None:
            break
        nd = 0 if first is None else int(np.count_nonzero(out != first))
        if first is None:
            first = out.copy()
        print(f"interp rep {r}: {hashlib.sha256(out.tobytes()).hexdigest()[:16]} differing words {nd}", flush=True)
    pr.close()


if __name__ == "__main__":
    main()
