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
import resource
import socket
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
LDE_ITERS = 110  # timed trace-LDE launch sets for the roofline (~160 ms at 2^16 x 8 x 64 proofs)


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


def _pinned(nbytes, device):
    import torch
    return torch.empty(nbytes, dtype=torch.uint8, pin_memory=device.type == "cuda")


class Exchange:
    """The exchange step of a sharded run (BASELINE configs[3]: 512 proofs over 8 GPUs; the reference's
    batch pattern is src/burn_mint_verifier.rs:326-338): rank 0 scatters each step's packed inputs,
    every rank proves its shard, rank 0 gathers the proofs.

    * inputs -- one scatter per step, issued `lookahead` steps before the step is submitted, then a
      D2H of the shard into a pinned ring slot; the submission waits for that job, long done by then;
    * proofs -- every rank's batch is proven straight into a fixed-size pinned record (int64 lengths,
      then one xfg_proof_size_bound slot per proof: no packing copy, no size all-reduce). Once the
      batch is done the record goes H2D, is gathered to rank 0 and the other ranks' rows are copied
      D2H into a pinned ring slot there; rank 0's own record never leaves the host (its proofs are
      read from the send record).

    Both run on one worker thread with its own process group and high-priority side stream, which
    sequences the steps on the HOST: a copy or collective is issued only once what it reads is
    complete, so no stream ever waits on another. A cross-stream wait is a barrier packet in one of
    the few hardware queues the prover's lane streams share, and it holds every lane kernel queued
    behind it until the other stream's work is done (round 4: with the collectives chained on the
    GPU the exchange cost 9-15 % of the proving throughput at world size 1). One worker, one group:
    the loop hands it scatters and gathers in step order, the same on every rank, so every rank
    issues the same sequence of collectives (two communicators driven from two threads could issue
    them in different orders on different ranks, and RCCL kernels waiting for peers behind each
    other in a hardware queue can deadlock). The proving loop only hands work over and, at the end,
    picks up the last gather.

    On the gloo backend (CPU rehearsal, tests/test_dist.py) the same steps run on host tensors and
    the collectives' Work handles are waited for directly."""

    def __init__(self, rank, world, per, cap, device, dist, send_slots, recv_slots=4, lookahead=4, emulate=0):
        import queue
        import threading
        import torch
        self.rank, self.world, self.per, self.cap = rank, world, per, cap
        self.device, self.dist, self.cuda = device, dist, device.type == "cuda"
        self.hdr = 8 * per
        self.rec = self.hdr + per * cap
        # records rank 0 receives per step: one per rank, or `emulate` at world size 1 (bench.py
        # --emulate-ranks K: the load of rank 0 at N = K -- one RCCL gather per step that receives K
        # real-size records, and the D2H of the K - 1 "peer" rows; those rows are copies of the first
        # record this rank sent, standing in for the peers' proofs)
        self.rows = emulate if emulate > 1 and world == 1 and self.cuda else world
        opts = None
        if self.cuda and hasattr(dist, "ProcessGroupNCCL"):
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True  # RCCL's own streams off the lanes' hardware queues
        mk = getattr(dist, "new_group", None)
        self.group = mk(pg_options=opts) if mk else None
        if self.group is not None:
            dist.barrier(group=self.group)  # the communicator is set up here, not in the timed steps
        self.side = torch.cuda.Stream(device, priority=-1) if self.cuda else None
        self.send = [_pinned(self.rec, device) for _ in range(send_slots)]
        self.send_busy = [None] * send_slots  # the gather job that last read the slot
        self.send_owned = [False] * send_slots  # claimed by a batch that has not been gathered yet
        self.next_send = 0
        # one device record each way (emulated: the K-row contribution): the gather worker runs one
        # gather at a time
        self.send_dev = torch.empty(self.rec * (self.rows // world), dtype=torch.uint8, device=device) \
            if self.cuda else None
        self.peer_rows_set = False
        self.next_recv, self.recv_slots = 0, recv_slots
        if rank == 0:
            self.recv_host = [_pinned(self.rows * self.rec, device).view(self.rows, self.rec)
                              for _ in range(recv_slots)]
            self.recv_dev = torch.empty((self.rows, self.rec), dtype=torch.uint8, device=device) if self.cuda else None
            # device path: the other rows' length headers and the longest proof of each gather
            # (_pack_d2h); the ring slot then holds the packed [rows - 1, per, maxlen] block
            self.recv_hdr = [_pinned((self.rows - 1) * self.hdr, device).view(self.rows - 1, self.hdr)
                             for _ in range(recv_slots)] if self.cuda and self.rows > 1 else None
            self.packed_len = [0] * recv_slots
        self.d2h_bytes_last = 0
        self.lookahead = max(1, lookahead)
        ring = self.lookahead + 1
        self.in_host = [_pinned(per * REC, device).view(per, REC) for _ in range(ring)]
        self.in_dev = torch.empty((per, REC), dtype=torch.uint8, device=device) if self.cuda else None
        self.in_pending = [None] * ring
        self.packed, self.nsteps = None, 0
        self.blocked = 0.0  # loop seconds spent waiting for exchange jobs (XFG_BENCH_PHASES)
        self.jobs = queue.Queue()
        self.worker = threading.Thread(target=self._work, args=(self.jobs,), daemon=True)
        self.worker.start()

    def _work(self, q):
        import torch
        if self.cuda:
            torch.cuda.set_device(self.device)
        while True:
            job = q.get()
            if job is None:
                return
            fn, done = job
            try:
                fn()
            except BaseException as e:  # surfaced by the loop's wait on `done`
                done.err = e
            done.ev.set()

    def _submit(self, fn):
        job = _Job()
        self.jobs.put((fn, job))
        return job

    def _done(self, job):
        if job is None:
            return
        t = time.perf_counter()
        job.wait()
        self.blocked += time.perf_counter() - t

    def _coll(self, stream, op, *args, **kw):
        """issue a collective from `stream` and wait for it on the host only (Work.wait() would
        make the stream wait on RCCL's stream on the GPU)"""
        import torch
        if not self.cuda:
            op(*args, async_op=True, **kw).wait()
            return
        with torch.cuda.stream(stream):
            w = op(*args, async_op=True, **kw)
        while not w.is_completed():  # also true once the collective has failed
            time.sleep(2e-5)
        with torch.cuda.stream(stream):
            w.wait()  # raises a failed collective's error; the stream wait it adds is already satisfied

    def _copy(self, stream, dst, src):
        import torch
        with torch.cuda.stream(stream):
            dst.copy_(src, non_blocking=True)
        stream.synchronize()

    def close(self):
        self.jobs.put(None)
        self.worker.join()

    # ---- inputs
    def start_inputs(self, packed, nsteps):
        """`packed`: rank 0's list of [world, per, REC] uint8 tensors, one per step (resident in HBM
        before the timed region), None elsewhere. Issues the first `lookahead` scatters."""
        self.packed, self.nsteps = packed, nsteps
        for i in range(min(self.lookahead, nsteps)):
            self._scatter(i)

    def _scatter(self, i):
        slot = i % len(self.in_pending)
        if self.in_pending[slot] is not None:  # the slot's previous scatter (rank 0 took its own shard
            self._done(self.in_pending[slot][1])  # locally and did not wait for it): long done by now
        chunks = list(self.packed[i].unbind(0)) if self.rank == 0 else None

        def job():
            dst = self.in_dev if self.cuda else self.in_host[slot]
            self._coll(self.side, self.dist.scatter, dst, chunks, src=0, group=self.group)
            if self.cuda:
                self._copy(self.side, self.in_host[slot], self.in_dev)
        self.in_pending[slot] = (i, self._submit(job))

    def inputs(self, i, local=None):
        """step i's shard as prove kwargs (issues step i + lookahead's scatter). `local`: the root's own
        shard, which it holds already (rank 0 proves it without waiting for its chunk of the scatter --
        the scatter still runs for the peers, as MPI's root keeps its own chunk)"""
        slot = i % len(self.in_pending)
        j, h = self.in_pending[slot]
        assert j == i, (j, i)
        if local is None:
            self._done(h)
            kws = unpack_inputs(self.in_host[slot].numpy())
            self.in_pending[slot] = None
        else:
            kws = local
        if i + self.lookahead < self.nsteps:
            self._scatter(i + self.lookahead)
        return kws

    # ---- proofs
    def claim(self):
        """a free send record for the next batch: (slot, host address, bytes, owning tensor)"""
        s = self.next_send
        if self.send_owned[s]:
            raise RuntimeError("Exchange: more batches in flight than send records")
        self.next_send = (s + 1) % len(self.send)
        self._done(self.send_busy[s])
        self.send_busy[s] = None
        self.send_owned[s] = True
        return s, self.send[s].data_ptr(), self.rec, self.send[s]

    def gather(self, s):
        """record s holds a complete batch: send it to rank 0 (asynchronous); returns a Gathered,
        whose proofs stay valid until recv_slots later gathers reuse its ring slot"""
        r = None
        if self.rank == 0:
            r = self.next_recv
            self.next_recv = (r + 1) % self.recv_slots

        def job():
            import torch
            if self.cuda:
                # rank 0's own record is already in its host memory: it is not copied to the device
                # (its gather contribution is whatever send_dev holds) nor back, Gathered.proofs reads
                # it from the send record; only the other rows come back D2H. Emulated ranks do copy
                # it up: the rows standing in for the peers are copies of it
                emul = self.rows != self.world
                if self.rank != 0 or emul:
                    self._copy(self.side, self.send_dev[:self.rec], self.send[s])
                if emul and not self.peer_rows_set:  # once: the peer rows' content (device copies)
                    with torch.cuda.stream(self.side):
                        self.send_dev.view(self.rows, self.rec)[1:].copy_(
                            self.send_dev[:self.rec].expand(self.rows - 1, self.rec))
                    self.side.synchronize()
                    self.peer_rows_set = True
                got = [self.recv_dev.view(-1)] if emul else (list(self.recv_dev.unbind(0)) if self.rank == 0 else None)
                self._coll(self.side, self.dist.gather, self.send_dev, got, dst=0, group=self.group)
                if self.rank == 0 and self.rows > 1:
                    self._pack_d2h(r)
            else:
                got = list(self.recv_host[r].unbind(0)) if self.rank == 0 else None
                self._coll(None, self.dist.gather, self.send[s], got, dst=0, group=self.group)
        h = self._submit(job)
        self.send_busy[s] = h
        self.send_owned[s] = False
        return Gathered(self, h, r, s)

    def _pack_d2h(self, r):
        """rank 0, after a gather: bring the other rows' proofs to the host packed. The rows' length
        headers come first (a few KB); every proof slot of the gathered records is then cut to the
        longest proof actually present and the [rows - 1, per, maxlen] block is packed on the device
        (one copy kernel on the side stream) and copied D2H -- instead of the records' full
        proof-size-bound slots (each sized for the worst-case opening)"""
        import numpy as np
        rows = self.rows - 1
        hdr = self.recv_hdr[r]
        self._copy(self.side, hdr, self.recv_dev[1:, :self.hdr])
        lens = hdr.numpy().view(np.int64)
        maxlen = int(min(max(int(lens.max()), 0), self.cap))
        self.packed_len[r] = maxlen
        if maxlen:
            # (measured against the full-row D2H: equal within noise at the emulated N = 8 load, and
            # one hipMemcpy2DAsync per row instead of the copy kernel -30 %: profiles/r06/exchange_x8.txt)
            src = self.recv_dev[1:, self.hdr:].view(rows, self.per, self.cap)[:, :, :maxlen]
            dst = self.recv_host[r].view(-1)[:rows * self.per * maxlen].view(rows, self.per, maxlen)
            self._copy(self.side, dst, src)
        self.d2h_bytes_last = rows * self.hdr + rows * self.per * maxlen

    def drain(self):
        for h in self.send_busy + [p[1] for p in self.in_pending if p]:
            self._done(h)


class _Job:
    """completion of an exchange job run by a worker thread"""

    def __init__(self):
        import threading
        self.ev = threading.Event()
        self.err = None

    def wait(self):
        self.ev.wait()
        if self.err is not None:
            raise self.err


class Gathered:
    """one step's gathered proofs on rank 0 (a handle on the asynchronous exchange)"""

    def __init__(self, ex, h, slot, send_slot):
        self.ex, self.h, self.slot, self.send_slot = ex, h, slot, send_slot

    def proofs(self):
        """waits for the exchange; rank 0: all ranks' proofs in rank order, zero-copy memoryviews
        into the pinned ring slot and, for rank 0's own proofs, into its send record (valid until the
        slot is reused, recv_slots gathers later, and the record is claimed again, send_slots batches
        later); None elsewhere. A zero or oversized length (a failed proof) raises."""
        import numpy as np
        ex = self.ex
        ex._done(self.h)
        if self.slot is None:
            return None
        allb = ex.recv_host[self.slot].numpy()
        out = []
        for q in range(ex.rows):
            if q == 0 and ex.cuda:
                # rank 0's own record never left its host memory: read it from the send record
                row = ex.send[self.send_slot].numpy()
                lens, body, slot = row[:ex.hdr].view(np.int64), row[ex.hdr:], ex.cap
            elif ex.cuda:  # packed by _pack_d2h: headers apart, slots cut to the longest proof
                slot = ex.packed_len[self.slot]
                lens = ex.recv_hdr[self.slot][q - 1].numpy().view(np.int64)
                body = allb.reshape(-1)[(q - 1) * ex.per * slot:q * ex.per * slot]
            else:
                row = allb[q]
                lens, body, slot = row[:ex.hdr].view(np.int64), row[ex.hdr:], ex.cap
            mv = memoryview(body)
            for i, ln in enumerate(lens):
                if not 0 < ln <= min(slot, ex.cap):
                    raise RuntimeError(f"exchange: rank {q} proof {i} has no proof in its record (length {ln})")
                out.append(mv[i * slot:i * slot + int(ln)])
        return out


def pipelined_steps(submit_fn, collect_fn, batches, depth=2, ex=None, packed=None):
    """run len(batches) steps with `depth` batches in flight: step i+depth-1 is submitted before step
    i's proofs are collected, so the host tail of one batch (and the collection) overlaps the kernels
    of the next ones. Every step is proven in full. Single process (ex None): submit_fn(kws) ->
    pending, collect_fn(pending) -> proofs; returns the last step's proofs. Sharded (ex an Exchange):
    each step's shard comes from its own scatter, submit_fn(kws, record) proves into an exchange
    record and the completed record is gathered to rank 0; returns the last step's proofs on rank 0,
    None elsewhere, after every exchange of the window has completed."""
    pending, out, failed = [], None, []
    tl = [] if os.environ.get("XFG_BENCH_TIMELINE") else None  # step completion times (stderr)
    ts = []
    # XFG_BENCH_PHASES=1: host time of the loop's phases (scatter, submit, wait, gather), stderr
    ph = {"scatter": 0.0, "submit": 0.0, "wait": 0.0, "gather": 0.0} if os.environ.get("XFG_BENCH_PHASES") else None
    clk = time.perf_counter

    def collect(item):
        p, s = item
        t1 = clk()
        if ex is None:
            got = collect_fn(p)
            if ph is not None and hasattr(p, "wait"):
                p.wait()
            t2 = clk()
        else:
            try:
                p.record_ready()  # the batch is complete in its record (raises on a failed proof)
            except Exception as e:
                # the failed proof's length is zeroed in the record, which still travels: every rank
                # keeps issuing the same collectives (raising here would leave the peers waiting in
                # this gather until the RCCL timeout); raised once the window's exchanges are done
                failed.append(e)
            t2 = clk()
            got = ex.gather(s)
        if ph is not None:
            ph["wait"] += t2 - t1
            ph["gather"] += clk() - t2
        return got

    t0 = clk()
    if ex is not None:
        ex.blocked = 0.0
        ex.start_inputs(packed, len(batches))
    for i, b in enumerate(batches):
        t1 = clk()
        s, rec = None, None
        if ex is not None:
            b = ex.inputs(i, b[:ex.per] if ex.rank == 0 and b is not None else None)
            s, addr, nbytes, owner = ex.claim()
            rec = (addr, nbytes, owner)
        t2 = clk()
        pending.append((submit_fn(b) if rec is None else submit_fn(b, rec), s))
        if ph is not None:
            ph["scatter"] += t2 - t1
            ph["submit"] += clk() - t2
        if tl is not None:
            ts.append(clk() - t0)
        if len(pending) >= depth:
            out = collect(pending.pop(0))
            if tl is not None:
                tl.append(clk() - t0)
    while pending:
        out = collect(pending.pop(0))
        if tl is not None:
            tl.append(clk() - t0)
    if ex is not None:
        t1 = clk()
        try:
            out = out.proofs() if out is not None else None
        finally:
            ex.drain()
        if failed:
            raise failed[0]
        if ph is not None:
            ph["gather"] += clk() - t1
    if tl:
        print("timeline ms: " + " ".join(f"{t * 1e3:.1f}" for t in tl), file=sys.stderr)
        print("submitted ms: " + " ".join(f"{t * 1e3:.1f}" for t in ts), file=sys.stderr)
    if ph is not None:
        print("phases ms: " + " ".join(f"{k}={v * 1e3:.1f}" for k, v in ph.items()) +
              f" total={(clk() - t0) * 1e3:.1f}" +
              (f" (of which waiting on earlier exchanges {ex.blocked * 1e3:.1f})" if ex is not None else ""),
              file=sys.stderr)
    return out


def config5(prover, gpu, batch=4, calls=12, depth=6):
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
        # of a single proof, each over a window of >= 150 ms of back-to-back launch sets (as LDE_ITERS)
        lde_ms = prover.bench_lde(batch, n5, 16, 36)
        lde1_ms = prover.bench_lde(1, n5, 16, 140)
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


def single_proof(prover, n, reps=10, source=0):
    """latency of one proof (BASELINE configs[1] at n = 2^16): xfg_prove_burn_mint called
    synchronously, best of `reps` after one warm call, and the library's stage split of one more call
    (XFG stage timers: host marshalling, each GPU stage, host replay and serialisation)"""
    kw = synthetic.burn_inputs(source)
    prover.prove_burn_mint(**kw, trace_length=n)
    times = []
    for _ in range(reps):
        t = time.perf_counter()
        prover.prove_burn_mint(**kw, trace_length=n)
        times.append((time.perf_counter() - t) * 1e3)
    prover.set_timing(True)
    prover.prove_burn_mint(**kw, trace_length=n)
    stages = {k: round(v, 3) for k, v in prover.stage_times().items()}
    prover.set_timing(False)
    return {"workload": f"configs[1]: one burn proof, {n}-step trace, blowup {BLOWUP}, xfg_prove_burn_mint "
                        "(synchronous)", "ms": round(min(times), 3), "median_ms": round(sorted(times)[reps // 2], 3),
            "reps": reps, "stage_ms": stages}


def whole_proof_line(proofs_per_s, n, world):
    b = whole_proof_bytes(n, BLOWUP)
    achieved = proofs_per_s * b / 1e9
    return {"bytes_per_proof": b, "achieved_GBps": round(achieved, 1), "peak": PEAK_HBM_GBS * world,
            "frac": round(achieved / (PEAK_HBM_GBS * world), 4),
            "note": "SURVEY 8(d) whole-proof algorithmic bytes (each stage reads its inputs and writes its "
                    "outputs once) x proofs/s, against the HBM peak of all GPUs",
            "valu": whole_proof_valu(proofs_per_s, n, world)}


def whole_proof_valu(proofs_per_s, n, world):
    """the bound that holds for the whole proof: VALU issue. Lane instructions per proof from the
    committed ledger (profiles/rNN/valu_per_proof.json, scripts/valu_ledger.sh: SQ_INSTS_VALU of every
    kernel, 3 minus 1 pipelined batches) x proofs/s, against the half-rate issue ceiling of all GPUs"""
    import glob
    if n != 1 << LOG_N:
        return None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "valu_per_proof.json")), reverse=True):
        d = json.load(open(f))
        rate = d["lane_instr_per_proof"] * proofs_per_s / 1e12
        # the ceiling of the proof's instruction mix (scripts/valu_ceiling.py: measured issue rate per
        # instruction form over each kernel's ISA, weighted by its share), else the half-rate class
        ceil = d.get("ceiling_T_lane_instr_s", VALU_HALF_RATE_T) * world
        return {"lane_instr_per_proof": d["lane_instr_per_proof"], "achieved_T_lane_instr_s": round(rate, 2),
                "ceiling_T_lane_instr_s": ceil, "frac": round(rate / ceil, 3), "source": os.path.relpath(f, ROOT)}
    return None


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


VALU_HALF_RATE_T = 36.0  # measured issue rate of the 64-bit / carry / three-source VALU forms the field code is
#                          made of (profiles/r05/valu_ubench.txt; the LDE passes' mix ceiling is 37.0)


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


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(gpus, argv, limit_s=None):
    """`bench.py --gpus N` (N > 1) without a launcher: start N ranks with torch.distributed.run as a
    CHILD process (this process never touches the GPU, so nothing is exec'd from a GPU-initialised
    process), relay rank 0's JSON line to stdout and everything else to stderr, and return the child's
    exit code. The child runs in its own process group: if this process is interrupted, or the ranks
    outlive `limit_s` seconds (XFG_BENCH_LIMIT_S, default none), the whole group is terminated (then
    killed) and a non-zero code returned, so no torchrun or rank is left behind. Reference harness:
    src/benchmarks/mod.rs:301-342."""
    import signal
    import subprocess
    import threading
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1, start_new_session=True)
    expired = threading.Event()

    def stop():
        if p.poll() is not None:
            return
        for sig, wait in ((signal.SIGTERM, 15), (signal.SIGKILL, 15)):
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                return
            try:
                p.wait(timeout=wait)
                return
            except subprocess.TimeoutExpired:
                pass

    def expire():
        expired.set()
        stop()
    limit_s = limit_s if limit_s is not None else float(os.environ.get("XFG_BENCH_LIMIT_S", "0"))
    timer = threading.Timer(limit_s, expire) if limit_s > 0 else None
    if timer is not None:
        timer.daemon = True
        timer.start()
    try:
        for line in p.stdout:
            print(line, end="", file=sys.stdout if line.lstrip().startswith("{") else sys.stderr, flush=True)
        rc = p.wait()
    finally:
        if timer is not None:
            timer.cancel()
        stop()
    if expired.is_set():
        print(f"bench.py: ranks still running after {limit_s:.0f} s, terminated", file=sys.stderr)
        return rc or 124
    return rc


def rank_cpus(local_rank, local_world, cpus):
    """the host CPUs of one rank when `local_world` ranks share this node: a disjoint, contiguous slice
    of the CPUs this process may run on (`cpus`), so the ranks' lane workers and host pools do not
    migrate across each other; all of `cpus` when there are fewer CPUs than ranks"""
    cpus = sorted(cpus)
    k = len(cpus) // max(1, local_world)
    if local_world <= 1 or k == 0:
        return cpus
    return cpus[local_rank * k:(local_rank + 1) * k]


def parse_cpulist(text):
    """sysfs cpulist ("0-63,128-191") -> set of CPU ids"""
    out = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    return out


def gpu_local_cpus(index, sysfs="/sys", env=None):
    """the CPUs local to GPU `index` of this process's device order: the GPU nodes of the KFD topology
    this process may open, in topology order (the order ROCr enumerates them), narrowed by
    ROCR_VISIBLE_DEVICES and then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (index lists into the
    previous list), modulo the count (ranks sharing a GPU in a rehearsal) -> that PCI device's
    local_cpulist. None when the topology is not readable or a visibility list is not plain indices"""
    env = os.environ if env is None else env
    base = os.path.join(sysfs, "class", "kfd", "kfd", "topology", "nodes")
    try:
        gpus = []
        for d in sorted(os.listdir(base), key=int):
            try:  # a GPU this process may not open (a shared box's other cards) is not one of its devices
                with open(os.path.join(base, d, "properties")) as f:
                    props = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
            except PermissionError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                gpus.append(props)
        for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
            if env.get(var):
                gpus = [gpus[int(i)] for i in env[var].split(",")]
        p = gpus[index % len(gpus)]
        loc, dom = int(p["location_id"]), int(p.get("domain", "0"))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 31:02x}.{loc & 7:x}"
        with open(os.path.join(sysfs, "bus", "pci", "devices", bdf, "local_cpulist")) as f:
            return parse_cpulist(f.read()) or None
    except (OSError, ValueError, KeyError, IndexError, ZeroDivisionError):
        return None


def rank_cpus_local(local_rank, local_world, cpus, local_sets):
    """NUMA-aware rank_cpus: the ranks whose GPUs share a set of local CPUs split that set (within the
    CPUs this process may use) between them, so every rank's host threads -- which fill the pinned
    host blocks its GPU reads and writes directly -- sit next to its GPU; rank_cpus when any rank's
    local set is unknown or too small for the ranks that share it"""
    cpus = set(cpus)
    if local_world <= 1 or any(ls is None for ls in local_sets):
        return rank_cpus(local_rank, local_world, cpus)
    mine = local_sets[local_rank]
    peers = [r for r in range(local_world) if local_sets[r] == mine]
    pool = sorted(mine & cpus)
    k = len(pool) // len(peers)
    if k == 0:
        return rank_cpus(local_rank, local_world, cpus)
    i = peers.index(local_rank)
    return pool[i * k:(i + 1) * k]


def host_threads_for(ncpus):
    """XFG_HOST_THREADS for a rank with `ncpus` CPUs: the library's default 8 on a 16-CPU share (the
    other half runs the lane workers), fewer on a smaller share"""
    return max(2, min(8, ncpus // 2))


def pin_rank(env):
    """pin this rank (before torch or HIP start any thread) to its slice of the node's CPUs -- next to
    its GPU where the topology says which CPUs those are -- and size the library's host pool to it,
    unless the caller set XFG_HOST_THREADS; -> the slice"""
    if not hasattr(os, "sched_setaffinity"):
        return None
    local_world = int(env.get("LOCAL_WORLD_SIZE", env.get("WORLD_SIZE", "1")))
    local_rank = int(env.get("LOCAL_RANK", "0"))
    cpus = os.sched_getaffinity(0)
    mine = sorted(cpus)
    if local_world > 1:
        # NUMA-aware when the GPU topology is readable: on a two-socket node a contiguous slice by CPU
        # id would put half the ranks on the socket away from their GPU
        mine = rank_cpus_local(local_rank, local_world, cpus, [gpu_local_cpus(r, env=env) for r in range(local_world)])
        os.sched_setaffinity(0, mine)
        env.setdefault("XFG_HOST_THREADS", str(host_threads_for(len(mine))))
    return mine


def check_world(gpus, env):
    """under a launcher the world size is the launcher's: a --gpus that disagrees is an error, not a
    silent N = WORLD_SIZE run (the driver's 1 -> 8 curve reads n_gpus from the line)"""
    world = int(env.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in env and gpus != world:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    return world


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs = ranks; N > 1 without a launcher starts torch.distributed.run itself")
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
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="with --dist at world size 1: rank 0's gather receives this many real-size "
                         "records per step over RCCL (its own, then copies), as rank 0 does at N = this "
                         "(rehearses the N = 8 exchange load on one GPU)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = check_world(args.gpus, os.environ)
    cpus = pin_rank(os.environ)

    import torch
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
        # nccl: bind the communicator to this rank's GPU up front (without device_id RCCL guesses
        # the device from the global rank and warns that a wrong guess can hang)
        dist.init_process_group(backend, **({"device_id": torch.device("cuda", gpu)} if backend == "nccl" else {}))
    device = torch.device("cuda", gpu) if backend == "nccl" else torch.device("cpu")

    import xfgstark
    prover = xfgstark.XfgBurnMintProver(device=gpu)
    n = 1 << args.log_n
    per = args.per_gpu
    # workspace allocation and code-object load (setup, not a proving step)
    prover.prepare(per, n, buffers=0)

    # synthetic inputs for every step, generated before the timed region (rank 0 holds the
    # batches; for N > 1 they are packed into HBM and each step's shard is scattered over RCCL)
    total_steps = args.warmup + args.steps
    batches = [[synthetic.burn_inputs(k * per * world + i) for i in range(per * world)] if rank == 0 else None
               for k in range(total_steps)]
    packed, ex = None, None
    if dist is not None:
        packed = [torch.from_numpy(pack_inputs(b)).to(device).view(world, per, REC) if rank == 0 else None
                  for b in batches]
        # the exchange's pinned records and device buffers (setup): one send record per batch in
        # flight plus the ones whose gathers may still run
        ex = Exchange(rank, world, per, prover.proof_size_bound(n), device, dist, send_slots=args.depth + 3,
                      emulate=args.emulate_ranks)

    # single process: every batch is proven straight into one of a ring of host records (int64 lengths,
    # then one proof-size-bound slot per proof), as the sharded path proves into its exchange records;
    # a step's proofs are then zero-copy views of its record -- no per-proof bytes objects are built
    # inside the timed window (the ring has a record for every batch in flight, plus the last step's)
    import numpy as np
    ring = [] if dist is not None else [np.ones(8 * per + per * prover.proof_size_bound(n), dtype=np.uint8)
                                        for _ in range(args.depth + 2)]
    ring_next = [0]

    def submit_fn(kws, record=None):
        if record is None:
            r = ring[ring_next[0] % len(ring)]
            ring_next[0] += 1
            record = (r.ctypes.data, r.size, r)
        addr, nbytes, owner = record  # the exchange's record (sharded) or the ring's
        return prover.submit_batch_record(kws, n, addr, nbytes, owner=owner)

    def collect_fn(pending):
        pending.record_ready()  # raises on a failed proof
        return pending.record_views()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(gpu)

    if args.warmup:
        pipelined_steps(submit_fn, collect_fn, batches[:args.warmup], args.depth, ex,
                        packed[:args.warmup] if packed else None)
    barrier()
    prover.lde_probe(True)  # HIP events around every trace-LDE launch set inside the timed steps
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    out = pipelined_steps(submit_fn, collect_fn, batches[args.warmup:], args.depth, ex,
                          packed[args.warmup:] if packed else None)
    barrier()
    el = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    # this rank's host load over the timed window: CPU seconds (all threads) per step and per second
    mine = {"rank": rank, "device": gpu, "host": socket.gethostname(), "cpus": len(cpus) if cpus else None,
            "cpu_first": min(cpus) if cpus else None,
            "host_threads": int(os.environ.get("XFG_HOST_THREADS", "8")),
            "cpu_s_per_step": round((ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime) / args.steps, 5),
            "cpu_util": round((ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime) / el, 2)}
    ranks = [mine]
    if dist is not None:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    if os.environ.get("XFG_BENCH_TIMELINE"):  # the window in the profiler's clock (CLOCK_MONOTONIC ns)
        print(f"window ns: {int(t0 * 1e9)} {int((t0 + el) * 1e9)}", file=sys.stderr)
    el_t = torch.tensor([el], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    pipe_ms, pipe_sets, pipe_polys = prover.lde_probe(False)
    verified = None
    if rank == 0:
        last = [bytes(x) for x in out]
        if ex is not None and ex.rows != world:  # emulated ranks: the stand-in peer rows
            peer = last[per:2 * per]
            assert len(last) == ex.rows * per and all(last[q * per:(q + 1) * per] == peer for q in range(1, ex.rows))
            last = last[:per]
        assert len(last) == per * world
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

    if ex is not None:
        ex.close()
    if rank != 0:  # the side measurements below are rank 0's
        prover.close()
        dist.barrier()
        dist.destroy_process_group()
        return

    # one synchronous batch call (no pipelining), for reference
    t = time.perf_counter()
    prover.prove_batch(batches[-1][:per], trace_length=n)
    sync_call_ms = (time.perf_counter() - t) * 1e3

    # BASELINE configs[1]: ONE proof of this shape through xfg_prove_burn_mint, synchronous (the
    # reference's prove_burn_mint, src/burn_mint_prover.rs:62-129): best of 10 after a warm call
    single = single_proof(prover, n)

    # ---- roofline: trace LDE kernel pair, algorithmic bytes 8*w*(n+N) per proof, timed over a window
    # of >= 150 ms of back-to-back launch sets: the chip's clock settles only after ~30 ms of load
    # (profiles/r04/lde_ramp.txt), so a short window mostly measures the transient
    lde_ms = prover.bench_lde(per, n, BLOWUP, LDE_ITERS)
    lde_bytes = 8 * WIDTH * (n + n * BLOWUP) * per
    achieved = lde_bytes / (lde_ms * 1e-3) / 1e9
    pmc, traffic_src = pmc_record(per, n, BLOWUP)
    traffic = pmc["traffic_bytes"] if pmc else None
    prover.set_timing(True)
    prover.prove_batch([synthetic.burn_inputs(i) for i in range(per)], trace_length=n)
    prover_stage = {k: round(v, 3) for k, v in prover.stage_times().items()}
    prover.set_timing(False)
    vrate = verify_rate(prover, last[:per], batches[-1][:per])
    c5 = None if args.no_config5 else config5(prover, gpu)

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
        # the exchange step of a sharded run (--dist / N > 1): one scatter of packed inputs per
        # step and one gather of fixed-size proof records per step, both inside the timed steps
        "exchange": None if ex is None else {
            "backend": backend, "scatter": f"one per step, issued {ex.lookahead} steps ahead",
            "gather": "one per step: fixed record of 8 B lengths + proof-size-bound slots per rank",
            "sequencing": "one host worker thread (own process group, high-priority streams), "
                          "collectives in step order; no cross-stream waits on the GPU",
            "record_bytes_per_rank": ex.rec, "proof_size_bound": ex.cap,
            "records_received_per_step": ex.rows,
            # what the collectives saw: the world size and every rank's (rank, device, host) as
            # all-gathered over the process group, and the bytes rank 0 copied D2H per step
            "world": world, "ranks": [[r["rank"], r["device"], r["host"]] for r in ranks],
            "d2h_bytes_per_step": ex.d2h_bytes_last, "d2h_bytes_unpacked": (ex.rows - 1) * ex.rec},
        # every rank's host CPU over the timed window (getrusage, all threads): whether the host was
        # the limit of a rank (cpu_util near its `cpus`)
        "host_load": ranks,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     # the kernel is VALU-issue-bound: the same launch set
                     # against the VALU ceiling, instruction counts from the same PMC record
                     "valu": valu_roofline(pmc, lde_ms, WIDTH * per * n * BLOWUP),
                     "kernel": "trace LDE (ntt_pass_a_cos2 + ntt_pass_b_tq<8,8,4,split>), 7 columns x "
                               f"{per} proofs, {lde_ms:.3f} ms/launch-set, {lde_bytes} algorithmic B",
                     "window": f"{LDE_ITERS} back-to-back launch sets after one warm launch, HIP events",
                     # the same launch sets inside the timed pipelined steps (per XFG_UNIT-proof unit,
                     # sharing the GPU with the other lanes' kernels)
                     "in_pipeline": in_pipeline(pipe_ms, pipe_sets, pipe_polys, n)},
        "whole_proof": whole_proof_line(total / el, n, world),
        "verified": verified,
        "verify": vrate,
        "stage_ms_one_batch": prover_stage,
        "sync_prove_batch_ms": round(sync_call_ms, 3),
        "single_proof": single,
    }
    if c5:
        line["config5"] = c5
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    print(json.dumps(line), flush=True)
    prover.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
