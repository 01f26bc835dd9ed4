"""bench.py -- burn-proofs/sec of the MI355X STARK prover (BASELINE.json metric).

One step = one batch of PER_GPU burn proofs per GPU (2^16-step trace, blowup 8, the reference's
ProofOptions 42/8/4/None/8/31): BASELINE configs[2] at N=1, configs[3] (512 proofs on 8 GPUs)
at N=8. Rank 0 holds the batch inputs and the proofs: it scatters packed inputs to the ranks and
gathers the proof bytes back over RCCL (torch.distributed "nccl" backend), the only exchange
step of the path; each rank proves its shard with libxfgstark.so (weak scaling).

Prints ONE JSON line (rank 0) with `roofline` (trace-LDE kernel pair, HIP-event timed on the
prover's stream), `whole_proof` (SURVEY 8(d)'s per-proof algorithmic bytes x proofs/s against the
HBM peak), `verified` (every proof of the last timed step, gathered on rank 0, accepted by the GPU
batch verifier against its statement -- the run fails otherwise), `verify` (batch-verify
throughput, GPU vs host threads) and `cpu_baseline` (the oracle C restatement on the host cores:
1 thread in the reference-faithful per-row Keccak mode, and all cores with OpenMP).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "xfg-stark_amd"))
sys.path.insert(0, ROOT)

import synthetic  # noqa: E402

LOG_N = 16
BLOWUP = 8
WIDTH = 7
REC = 128  # packed input record bytes
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def pack_inputs(kws):
    """[count, REC] uint8 records: burn u64, mint u64, tx 32, recipient 20, secret 32, ids 3xu32"""
    import numpy as np
    out = np.zeros((len(kws), REC), dtype=np.uint8)
    for i, kw in enumerate(kws):
        b = bytearray()
        b += kw["burn_amount"].to_bytes(8, "little") + kw["mint_amount"].to_bytes(8, "little")
        b += kw["tx_prefix_hash"] + kw["recipient_address"].ljust(20, b"\0")[:20] + kw["secret"].ljust(32, b"\0")[:32]
        b += kw["network_id"].to_bytes(4, "little") + kw["target_chain_id"].to_bytes(4, "little")
        b += kw["commitment_version"].to_bytes(4, "little")
        out[i, :len(b)] = np.frombuffer(bytes(b), dtype=np.uint8)
    return out


def unpack_inputs(arr):
    res = []
    raw = arr.tobytes()  # one copy; records sliced from it
    for i in range(len(arr)):
        b = raw[i * REC:(i + 1) * REC]
        res.append(dict(burn_amount=int.from_bytes(b[0:8], "little"), mint_amount=int.from_bytes(b[8:16], "little"),
                        tx_prefix_hash=b[16:48], recipient_address=b[48:68], secret=b[68:100],
                        network_id=int.from_bytes(b[100:104], "little"),
                        target_chain_id=int.from_bytes(b[104:108], "little"),
                        commitment_version=int.from_bytes(b[108:112], "little")))
    return res


def scatter_all(batches, rank, world, per_rank, device, dist, packed=None):
    """every step's shard in ONE scatter (rank 0 holds all steps' inputs in HBM): [K, per_rank, REC]
    uint8 records of this rank on the host, unpacked per step by the caller. One collective per
    window instead of one per step -- a per-step scatter and the host sync on its shard waited
    ~0.8 ms per step for its RCCL kernel on a GPU the prover's lanes keep full"""
    import torch
    K = len(batches)
    if rank == 0:
        if packed is None:
            packed = [torch.from_numpy(pack_inputs(b)).to(device).view(world, per_rank, REC) for b in batches]
        big = torch.stack(list(packed[:K]), dim=1)  # [world, K, per_rank, REC]
        chunks = list(big.unbind(0))
    else:
        chunks = None
    local = torch.empty((K, per_rank, REC), dtype=torch.uint8, device=device)
    dist.scatter(local, chunks, src=0)
    return local.cpu().numpy()


def scatter_inputs(all_inputs, rank, world, per_rank, device, dist, packed=None):
    """rank 0's batch inputs -> this rank's shard (list of prove kwargs). `packed` = the batch
    already packed into a [world, per_rank, REC] uint8 device tensor on rank 0 (resident in HBM)."""
    import torch
    if dist is None:
        return all_inputs
    if rank == 0:
        if packed is None:
            packed = torch.from_numpy(pack_inputs(all_inputs)).to(device).view(world, per_rank, REC)
        chunks = list(packed.unbind(0))
    else:
        chunks = None
    local = torch.empty((per_rank, REC), dtype=torch.uint8, device=device)
    dist.scatter(local, chunks, src=0)
    return unpack_inputs(local.cpu().numpy())


class _Exchange:
    """reused buffers of gather_proofs: a pinned host record per rank (double-buffered, so a record
    is never rewritten while its host-to-device copy may still run), rank 0's device gather buffer
    and its pinned host copy"""
    send = None
    flip = 0
    big = None
    host = None


def _pinned(nbytes, device):
    import torch
    return torch.empty(nbytes, dtype=torch.uint8, pin_memory=device.type == "cuda")


def gather_proofs(proofs, rank, world, per_rank, device, dist):
    """this rank's proofs -> all proofs on rank 0 (None elsewhere) over the process group: one gather
    of [per_rank int64 lengths | concatenated proofs], padded to the longest rank record.
    `proofs` is a list of proof bytes or a submitted batch (xfgstark.PendingBatch), whose proofs
    are packed straight from the workers' output buffer into a pinned record. Rank 0 gathers into
    one reused device buffer, copies it to pinned host memory in one D2H and returns zero-copy
    memoryviews into it (valid until the next call)."""
    import numpy as np
    import torch
    if dist is None:
        return proofs
    X = _Exchange
    hdr = 8 * per_rank
    if hasattr(proofs, "packed_into"):
        cap = hdr + per_rank * proofs._cap
    else:
        cap = hdr + sum(len(p) for p in proofs)
    if X.send is None or X.send[0].numel() < cap:
        X.send = [_pinned(cap + (1 << 20), device), _pinned(cap + (1 << 20), device)]
    X.flip ^= 1
    rec = X.send[X.flip]
    buf = rec.numpy()
    if hasattr(proofs, "packed_into"):
        mine = proofs.packed_into(buf)
    else:
        lens = np.array([len(p) for p in proofs], dtype=np.int64)
        buf[:hdr] = lens.view(np.uint8)
        off = hdr
        for p in proofs:  # one copy of each proof, straight into the record
            buf[off:off + len(p)] = np.frombuffer(p, dtype=np.uint8)
            off += len(p)
        mine = off
    size = torch.tensor([mine], dtype=torch.int64, device=device)
    dist.all_reduce(size, op=dist.ReduceOp.MAX)
    size = int(size.item())
    t = rec[:size].to(device, non_blocking=True) if device.type == "cuda" else rec[:size]
    got = None
    if rank == 0:
        if X.big is None or X.big.shape[0] != world or X.big.shape[1] < size:
            X.big = torch.empty((world, size + (1 << 20)), dtype=torch.uint8, device=device)
        got = [X.big[r, :size] for r in range(world)]
    dist.gather(t, got, dst=0)
    if rank != 0:
        return None
    if device.type == "cuda":  # one D2H of all ranks' records into a reused pinned buffer
        if X.host is None or X.host.numel() < world * size:
            X.host = _pinned(world * size + (8 << 20), device)
        host = X.host[:world * size].view(world, size)
        host.copy_(X.big[:, :size])
        allb = host.numpy()
    else:
        allb = X.big[:, :size].numpy()
    out = []
    for r in range(world):
        row = allb[r]
        mv, off = memoryview(row), hdr
        for ln in row[:hdr].view(np.int64):
            out.append(mv[off:off + int(ln)])
            off += int(ln)
    return out


def sharded_step(prove_fn, all_inputs, rank, world, per_rank, device, dist):
    """scatter packed inputs from rank 0, prove the local shard, gather proof bytes to rank 0.
    Returns the list of proofs (bytes) on rank 0, None elsewhere."""
    local = scatter_inputs(all_inputs, rank, world, per_rank, device, dist)
    return gather_proofs(prove_fn(local), rank, world, per_rank, device, dist)


def pipelined_steps(submit_fn, collect_fn, batches, rank, world, per_rank, device, dist, packed=None, depth=2):
    """run len(batches) steps with `depth` batches in flight: every step's shard is scattered at the
    start (one collective), step i+depth-1 is submitted before step i's proofs are collected and
    gathered, so the host tail of one batch (and the Python collection) overlaps the kernels of the
    next ones. Every step is proven in full; returns the last step's proofs on rank 0."""
    pending, out = [], None
    tl = [] if os.environ.get("XFG_BENCH_TIMELINE") else None  # step completion times (stderr)
    ts = []
    # XFG_BENCH_PHASES=1: host time of the loop's phases (scatter, submit, wait, gather), stderr
    ph = {"scatter": 0.0, "submit": 0.0, "wait": 0.0, "gather": 0.0} if os.environ.get("XFG_BENCH_PHASES") else None
    clk = time.perf_counter

    def collect_gather(p):
        t1 = clk()
        got = collect_fn(p)
        if ph is not None and hasattr(p, "wait"):
            p.wait()
        t2 = clk()
        r = gather_proofs(got, rank, world, per_rank, device, dist)
        if ph is not None:
            ph["wait"] += t2 - t1
            ph["gather"] += clk() - t2
        return r

    t0 = clk()
    shards = scatter_all(batches, rank, world, per_rank, device, dist, packed) if (dist is not None and batches) else None
    for i, b in enumerate(batches):
        t1 = clk()
        local = unpack_inputs(shards[i]) if shards is not None else b
        t2 = clk()
        pending.append(submit_fn(local))
        if ph is not None:
            ph["scatter"] += t2 - t1
            ph["submit"] += clk() - t2
        if tl is not None:
            ts.append(clk() - t0)
        if len(pending) >= depth:
            out = collect_gather(pending.pop(0))
            if tl is not None:
                tl.append(clk() - t0)
    while pending:
        out = collect_gather(pending.pop(0))
        if tl is not None:
            tl.append(clk() - t0)
    if tl:
        print("timeline ms: " + " ".join(f"{t * 1e3:.1f}" for t in tl), file=sys.stderr)
        print("submitted ms: " + " ".join(f"{t * 1e3:.1f}" for t in ts), file=sys.stderr)
    if ph is not None:
        print("phases ms: " + " ".join(f"{k}={v * 1e3:.1f}" for k, v in ph.items()) +
              f" total={(clk() - t0) * 1e3:.1f}", file=sys.stderr)
    return out


def config5(prover, gpu, batch=4, calls=8, depth=4):
    """side measurement of BASELINE configs[4]: 2^20-step trace, blowup 16, 96-bit class options
    (quadratic extension, 24 queries, grinding 4), batches of `batch` proofs per call on this GPU,
    `depth` calls in flight; the trace LDE (7 columns, one proof) against the HBM roofline with
    SURVEY 8(d)'s B_LDE = 8 w (n + N) = 998,244,352 B, and the device memory the shape adds"""
    import torch
    import xfgstark
    n5 = 1 << 20
    o = xfgstark.ProofOptions.reference()
    o.field_extension, o.blowup_factor, o.num_queries = 2, 16, 24
    saved = prover._options
    prover._options = o
    free0 = torch.cuda.mem_get_info(gpu)[0]
    try:
        prover.prepare(batch, n5, buffers=depth)
        kws = [synthetic.burn_inputs(50_000 + i) for i in range(batch)]
        pend = []
        t = time.perf_counter()
        for _ in range(calls):
            pend.append(prover.submit_batch(kws, trace_length=n5))
            if len(pend) >= depth:
                pend.pop(0).result()
        while pend:
            res = pend.pop(0).result()
        dt = time.perf_counter() - t
        assert all(not isinstance(r, Exception) for r in res)
        used = free0 - torch.cuda.mem_get_info(gpu)[0]
        # the trace-LDE launch set as the configs[4] pipeline runs it (one call's `batch` proofs), and
        # of a single proof
        lde_ms = prover.bench_lde(batch, n5, 16, 5)
        lde1_ms = prover.bench_lde(1, n5, 16, 5)
    finally:
        prover._options = saved
    lde_b = 8 * WIDTH * (n5 + 16 * n5) * batch
    gbps = lde_b / (lde_ms * 1e-3) / 1e9
    pmc, src = pmc_record(batch, n5, 16)
    return {"workload": "configs[4]: 2^20-step trace, blowup 16, quadratic extension, 24 queries, grinding 4",
            "proofs_per_call": batch, "proofs_per_s": round(batch * calls / dt, 2),
            "ms_per_proof": round(dt / (batch * calls) * 1e3, 3), "proof_bytes": len(res[0]),
            "trace_lde_proofs": batch, "trace_lde_ms": round(lde_ms, 3), "trace_lde_bytes": lde_b,
            "trace_lde_GBps": round(gbps, 1), "trace_lde_frac": round(gbps / PEAK_HBM_GBS, 4),
            "trace_lde_1proof_ms": round(lde1_ms, 3),
            "trace_lde_1proof_frac": round(lde_b / batch / (lde1_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
            "trace_lde_traffic": pmc["traffic_bytes"] if pmc else None, "traffic_source": src,
            "device_bytes_added": int(used), "proofs_in_flight": batch * depth}


def whole_proof_line(proofs_per_s, n, world):
    b = whole_proof_bytes(n, BLOWUP)
    achieved = proofs_per_s * b / 1e9
    return {"bytes_per_proof": b, "achieved_GBps": round(achieved, 1), "peak": PEAK_HBM_GBS * world,
            "frac": round(achieved / (PEAK_HBM_GBS * world), 4),
            "note": "SURVEY 8(d) whole-proof algorithmic bytes (each stage reads its inputs and writes its "
                    "outputs once) x proofs/s, against the HBM peak of all GPUs"}


def in_pipeline(ms, sets, polys, n):
    if not sets:
        return None
    b = 8 * (n + n * BLOWUP) * polys
    return {"launch_sets": sets, "avg_ms": round(ms / sets, 4), "polys_per_set": polys // sets,
            "achieved_GBps": round(b / (ms * 1e-3) / 1e9, 1)}


def pmc_record(per, n, blowup):
    """the committed PMC record of the trace-LDE launch set (profiles/rNN/lde_pmc.json, made by
    scripts/profile_round.sh: FETCH_SIZE x2 + WRITE_SIZE and SQ_INSTS_VALU, separate rocprofv3 --pmc
    runs) and its path, or (None, None)"""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "lde_pmc*.json")), reverse=True):
        d = json.load(open(f))
        if (d.get("count"), d.get("n"), d.get("blowup")) == (per, n, blowup):
            return d, os.path.relpath(f, ROOT)
    return None, None


VALU_HALF_RATE_T = 36.0  # measured issue ceiling of the 64-bit / carry VALU forms (scripts/ubench/valu_ubench.hip)


def valu_roofline(rec, lde_ms, outputs):
    """the bound that actually holds for the NTT: VALU issue. Lane-instructions per output from the
    PMC wave-instruction counts (x64 lanes), and the achieved issue rate at the measured launch-set
    time against the half-rate ceiling the Goldilocks carry / 64-bit forms run at"""
    if not rec or not rec.get("valu_insts_pass_a"):
        return None
    lane_instr = 64.0 * (rec["valu_insts_pass_a"] + rec["valu_insts_pass_b"])
    rate = lane_instr / (lde_ms * 1e-3) / 1e12
    return {"lane_instr_per_output": round(lane_instr / outputs, 1), "achieved_T_lane_instr_s": round(rate, 2),
            "ceiling_T_lane_instr_s": VALU_HALF_RATE_T, "frac": round(rate / VALU_HALF_RATE_T, 3),
            "valu_busy_pct": [rec.get("valu_busy_pct_pass_a"), rec.get("valu_busy_pct_pass_b")]}


def whole_proof_bytes(n, beta, w=WIDTH, e=8, c=2, fold=8, rem_deg=31):
    """SURVEY.md 8(d) notes: per-proof algorithmic HBM bytes, every stage reading its inputs once and
    writing its outputs once (c = 2 composition columns as SURVEY prices it; 221.2 MB at configs[2])"""
    b, N, nce = 8, n * beta, c * n
    tot = 2 * b * w * n + b * w * (n + N) + (b * w * N + 32 * N) + 64 * N  # interpolate, LDE, leaves, tree
    tot += (b * w * nce + e * nce) + 2 * e * nce + e * c * (n + N) + (e * c * N + 32 * N) + 64 * N
    tot += (b * w + e * c) * n + e * n + e * (n + N)  # DEEP combine + DEEP LDE
    D = N
    while D > (rem_deg + 1) * beta:  # FRI layers
        tot += e * D + 32 * D // fold + 64 * D // fold + e * D // fold
        D //= fold
    return tot


def host_facts():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(seconds=10.0):
    """the oracle C restatement (oracle/liboracle.so) on this host's cores, two modes:
    (i) 1 thread, faithful per-row Keccak recomputation like the reference (src/burn_mint_air.rs:264,376;
    Winterfell built without `concurrent`) -- the reference-faithful figure, `value`;
    (ii) all cores (OMP_NUM_THREADS, else the CPUs this process may run on) with OpenMP, one proof per
    thread, Keccak constants hoisted. Each mode runs for about `seconds`; per-stage CPU ms per proof."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    n = 1 << LOG_N
    opts = O.options()

    def airs(base, k):
        out = []
        for i in range(k):
            kw = synthetic.burn_inputs(base + i)
            st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"],
                                        kw["recipient_address"], kw["secret"])
            assert st == 0
            out.append(air)
        return out

    def run(faithful, threads, per_call):
        done, used, stages, t0 = 0, 0, {}, time.perf_counter()
        while True:
            used, lens, sts, ms = O.prove_batch(airs(10_000 + done, per_call), n, opts, faithful, threads)
            assert not any(sts), sts
            done += per_call
            for k, v in ms.items():
                stages[k] = stages.get(k, 0.0) + v
            el = time.perf_counter() - t0
            if el >= seconds:
                return done, used, el, {k: round(v / done, 1) for k, v in stages.items()}

    d1, _, el1, st1 = run(True, 1, 1)
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    d2, used2, el2, st2 = run(False, threads, threads)
    return {"value": d1 / el1, "unit": "proofs/s", "cores": 1, "kind": "port",
            "sample": f"{d1} proofs (2^16 steps, blowup 8) by oracle/liboracle.so in {el1:.1f}s, 1 thread, "
                      "faithful per-row Keccak (src/burn_mint_air.rs:264,376)",
            "stage_cpu_ms_per_proof": st1,
            "all_cores": {"value": d2 / el2, "unit": "proofs/s", "cores": used2, "kind": "port",
                          "sample": f"{d2} proofs by oracle/liboracle.so (OpenMP, {used2} threads, one proof "
                                    f"per thread, Keccak constants hoisted) in {el2:.1f}s",
                          "stage_cpu_ms_per_proof": st2},
            "host": host_facts()}


def verify_proofs(prover, proofs, inputs):
    """every proof against the statement rebuilt from its inputs, on the GPU (xfg_verify_batch_gpu)
    -> number accepted"""
    import xfgstark
    items = [(bytes(p), xfgstark.air_consts(**kw)) for p, kw in zip(proofs, inputs)]
    return sum(xfgstark.XfgBurnMintVerifier().batch_verify(items, gpu=prover))


def verify_rate(prover, proofs, inputs, threads=16, reps=3):
    """side measurement, src/burn_mint_verifier.rs:326-408 batch verify: proofs/s of one batch through
    the GPU batch verifier and through the host verifier on `threads` threads (best of `reps`)"""
    import xfgstark
    items = [(bytes(p), xfgstark.air_consts(**kw)) for p, kw in zip(proofs, inputs)]
    v = xfgstark.XfgBurnMintVerifier()
    best = {}
    for name, kw in (("gpu", {"gpu": prover}), ("host", {"threads": threads})):
        for _ in range(reps):
            t = time.perf_counter()
            ok = v.batch_verify(items, **kw)
            dt = time.perf_counter() - t
            assert all(ok)
            best[name] = min(best.get(name, dt), dt)
    return {"proofs": len(items), "gpu_proofs_per_s": round(len(items) / best["gpu"], 1),
            "host_proofs_per_s": round(len(items) / best["host"], 1), "host_threads": threads}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--per-gpu", type=int, default=64)
    ap.add_argument("--log-n", type=int, default=LOG_N)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-config5", action="store_true", help="skip the configs[4] side measurement")
    ap.add_argument("--depth", type=int, default=6, help="batches in flight (pipelined submission)")
    ap.add_argument("--dist", action="store_true",
                    help="run the scatter / gather collectives even at world size 1 (exercises the RCCL "
                         "path on a one-GPU box; launch with torch.distributed.run); rank 0 then also "
                         "checks the gathered proofs byte for byte against a direct prove_batch")
    ap.add_argument("--dump-proofs", default=None,
                    help="rank 0 writes the last step's gathered proofs here (u32 LE length + bytes each)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # XFG_DIST_BACKEND=gloo rehearses the N > 1 path on a box with fewer GPUs than ranks: the ranks
    # share the visible GPUs round-robin and the scatter / gather tensors stay on the host
    backend = os.environ.get("XFG_DIST_BACKEND", "nccl")
    gpu = local_rank % max(1, torch.cuda.device_count()) if backend != "nccl" else local_rank
    if world > 1 or args.dist:
        import torch.distributed as dist
        torch.cuda.set_device(gpu)
        dist.init_process_group(backend)
    device = torch.device("cuda", gpu) if backend == "nccl" else torch.device("cpu")

    import xfgstark
    prover = xfgstark.XfgBurnMintProver(device=gpu)
    n = 1 << args.log_n
    per = args.per_gpu
    # workspace allocation, code-object load and one host output buffer per batch in flight (setup,
    # not a proving step)
    prover.prepare(per, n, buffers=args.depth)

    # synthetic inputs for every step, generated before the timed region (rank 0 holds the
    # batches; for N > 1 they are packed into HBM and scattered over RCCL inside each step)
    total_steps = args.warmup + args.steps
    batches = [[synthetic.burn_inputs(k * per * world + i) for i in range(per * world)] if rank == 0 else None
               for k in range(total_steps)]
    packed = None
    if dist is not None:
        packed = [torch.from_numpy(pack_inputs(b)).to(device).view(world, per, REC) if rank == 0 else None
                  for b in batches]

    def submit_fn(kws):
        return prover.submit_batch(kws, trace_length=n)

    def collect_fn(pending):
        if dist is not None:  # packed straight into the exchange record by gather_proofs
            return pending
        res = pending.result()
        for r in res:
            if isinstance(r, Exception):
                raise r
        return [r.to_bytes() for r in res]

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(gpu)

    if args.warmup:
        pipelined_steps(submit_fn, collect_fn, batches[:args.warmup], rank, world, per, device, dist,
                        packed[:args.warmup] if packed else None, args.depth)
    barrier()
    prover.lde_probe(True)  # HIP events around every trace-LDE launch set inside the timed steps
    t0 = time.perf_counter()
    out = pipelined_steps(submit_fn, collect_fn, batches[args.warmup:], rank, world, per, device, dist,
                          packed[args.warmup:] if packed else None, args.depth)
    barrier()
    el = time.perf_counter() - t0
    el_t = torch.tensor([el], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    pipe_ms, pipe_sets, pipe_polys = prover.lde_probe(False)
    verified = None
    if rank == 0:
        assert out is not None and len(out) == per * world
        last = [bytes(x) for x in out]
        if args.dump_proofs:
            with open(args.dump_proofs, "wb") as f:
                for p in last:
                    f.write(len(p).to_bytes(4, "little") + p)
        # every proof of the last timed step (all ranks' shards, gathered in rank order) against the
        # statement of the input it was scattered for: a sharding or ordering bug fails the run
        verified = verify_proofs(prover, last, batches[-1])
        if verified != len(last):
            raise SystemExit(f"bench: {len(last) - verified} of {len(last)} proofs of the last step rejected")
        if args.dist:  # the collective path's output: the gathered proofs of the last step, in order
            want = [p.to_bytes() for p in prover.prove_batch(batches[-1], trace_length=n)]
            assert last == want, "gathered proofs differ from a direct prove_batch"

    # one synchronous batch call (no pipelining), for reference
    t = time.perf_counter()
    prover.prove_batch(batches[-1][:per] if rank == 0 else [synthetic.burn_inputs(i) for i in range(per)],
                       trace_length=n)
    sync_call_ms = (time.perf_counter() - t) * 1e3

    # ---- roofline: trace LDE kernel pair, algorithmic bytes 8*w*(n+N) per proof
    lde_ms = prover.bench_lde(per, n, BLOWUP, 10)
    lde_bytes = 8 * WIDTH * (n + n * BLOWUP) * per
    achieved = lde_bytes / (lde_ms * 1e-3) / 1e9
    pmc, traffic_src = pmc_record(per, n, BLOWUP)
    traffic = pmc["traffic_bytes"] if pmc else None
    prover.set_timing(True)
    prover_stage = {}
    if rank == 0:
        prover.prove_batch([synthetic.burn_inputs(i) for i in range(per)], trace_length=n)
        prover_stage = {k: round(v, 3) for k, v in prover.stage_times().items()}
    prover.set_timing(False)
    vrate = verify_rate(prover, last[:per], batches[-1][:per]) if rank == 0 else None
    c5 = None if (args.no_config5 or rank != 0) else config5(prover, gpu)

    if rank == 0:
        total = per * world * args.steps
        line = {
            "metric": "burn-proofs/sec (2^16-step trace, blowup=8)",
            "value": total / el,
            "unit": "proofs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {
                "workload": f"batch of {per} burn proofs per GPU (configs[2]; configs[3] = 512 proofs on 8 GPUs)",
                "trace_length": n, "blowup": BLOWUP, "proof_options": "42/8/4/None/8/31",
                "proofs_per_step": per * world,
                "parallelism": f"dp{world} (independent proofs; RCCL scatter of inputs, gather of proof bytes)",
                "submission": f"pipelined, depth {args.depth} (xfg_prove_batch_submit / xfg_batch_wait)",
            },
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         # the kernel is VALU-issue-bound: the same launch set
                         # against the VALU ceiling, instruction counts from the same PMC record
                         "valu": valu_roofline(pmc, lde_ms, WIDTH * per * n * BLOWUP),
                         "kernel": "trace LDE (ntt_pass_a_cos2 + ntt_pass_b_tq<8,8,4,split>), 7 columns x "
                                   f"{per} proofs, {lde_ms:.3f} ms/launch-set, {lde_bytes} algorithmic B",
                         # the same launch sets inside the timed pipelined steps (per XFG_UNIT-proof unit,
                         # sharing the GPU with the other lanes' kernels)
                         "in_pipeline": in_pipeline(pipe_ms, pipe_sets, pipe_polys, n)},
            "whole_proof": whole_proof_line(total / el, n, world),
            "verified": verified,
            "verify": vrate,
            "stage_ms_one_batch": prover_stage,
            "sync_prove_batch_ms": round(sync_call_ms, 3),
        }
        if c5:
            line["config5"] = c5
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(line), flush=True)
    prover.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
