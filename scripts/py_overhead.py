import sys, os, time, ctypes as C
if os.environ.get("WITH_TORCH") == "1":
    import torch
    torch.cuda.synchronize()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd")); sys.path.insert(0, ROOT)
import xfgstark, synthetic
pr = xfgstark.XfgBurnMintProver()
n = 1 << 16
for it in range(4):
    t0 = time.perf_counter()
    kws = [synthetic.burn_inputs(1000 * it + i) for i in range(64)]
    t1 = time.perf_counter()
    k = len(kws)
    arr = (xfgstark._BurnInputs * k)()
    keep = []
    for i, kw in enumerate(kws):
        s = xfgstark.burn_inputs(**kw); keep.append(s._keep); arr[i] = s
    o = pr._options._c()
    cap = xfgstark._lib.xfg_proof_size_bound(n, C.byref(o))
    if getattr(pr, "_out_cap", 0) < cap * k:
        pr._out = C.create_string_buffer(cap * k); pr._out_cap = cap * k
    base = C.addressof(pr._out)
    outs = (xfgstark._u8p * k)(*[C.cast(base + i * cap, xfgstark._u8p) for i in range(k)])
    lens = (C.c_size_t * k)(*([cap] * k)); sts = (C.c_int * k)()
    t2 = time.perf_counter()
    st = xfgstark._lib.xfg_prove_batch(pr._ctx, k, arr, n, C.byref(o), outs, lens, sts)
    t3 = time.perf_counter()
    res = [C.string_at(base + i * cap, lens[i]) for i in range(k)]
    t4 = time.perf_counter()
    print(f"gen {1e3*(t1-t0):.2f} pack {1e3*(t2-t1):.2f} C {1e3*(t3-t2):.2f} unpack {1e3*(t4-t3):.2f} ms")
for it in range(4):
    kws = [synthetic.burn_inputs(5000 * it + i) for i in range(64)]
    t0 = time.perf_counter()
    res = pr.prove_batch(kws, trace_length=n)
    t1 = time.perf_counter()
    out = [r.to_bytes() for r in res]
    t2 = time.perf_counter()
    print(f"prove_batch {1e3*(t1-t0):.2f} to_bytes {1e3*(t2-t1):.2f} ms")
