"""Locate the first differing proof section between the GPU path and the oracle (debug aid)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "xfg-stark_amd"), ROOT):
    sys.path.insert(0, p)
import numpy as np
import oracle_lib as O, synthetic, xfgstark

def sections(b):
    off = 0
    out = {}
    out["context"] = b[0:20]; off = 20
    out["nuq"] = b[20:21]; off = 21
    cl = int.from_bytes(b[off:off+2], "little"); off += 2
    com = b[off:off+cl]; off += cl
    for i in range(cl // 32):
        out[f"commit{i}"] = com[32*i:32*i+32]
    return out

for n, beta in [(64, 8), (1024, 8)]:
    kw = synthetic.REFERENCE_PACKAGE
    st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"], kw["recipient_address"], kw["secret"])
    opts = O.options(blowup=beta)
    st, want, dbg = O.prove(air, n, opts, debug=True)
    pr = xfgstark.XfgBurnMintProver()
    o = xfgstark.ProofOptions.reference(); o.blowup_factor = beta; pr._options = o
    tr = np.frombuffer(bytes(O.build_trace(air, n)), dtype=np.uint64).reshape(7, n)
    got = pr.prove_trace(tr, list(air.pub), air.nullifier, air.commitment).to_bytes()
    a, b = sections(want), sections(got)
    for k in a:
        print(n, beta, k, "OK" if a[k] == b.get(k) else "DIFF", a[k][:8].hex(), (b.get(k) or b"")[:8].hex())
    print("oracle z", dbg.z, "ood", list(dbg.ood))
    # ood frame location: search oracle bytes for z-dependent OOD values
    import struct
    oo = struct.pack("<Q", dbg.ood[0])
    print("ood0 in gpu proof:", got.find(oo) >= 0, "hz in gpu proof:", got.find(struct.pack("<Q", dbg.ood[14])) >= 0)
    for i in range(14):
        print(" ood", i, got.find(struct.pack("<Q", dbg.ood[i])) >= 0)
