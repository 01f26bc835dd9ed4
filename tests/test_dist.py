"""Multi-GPU path on CPU: bench.py's exchange step (bench.Exchange + bench.pipelined_steps) over
torch.distributed gloo with world_size 2, 4 and 8 (the driver's 8-GPU shape).

Rank 0 holds the packed burn inputs; each step's shard is scattered by its own collective, every
rank "proves" its shard into a fixed-size exchange record (here: the product's host marshalling,
xfgstark.air_consts, serialised -- variable-length outputs), rank 0 gathers the records. The result
must equal proving the whole batch on one rank, in order (independent proofs shard with no
data-path collective besides the input scatter / output gather)."""
import ctypes as C
import os
import socket
import struct

import pytest
import torch.multiprocessing as mp

FAKE_CAP = 400  # record slot of a fake proof (at most 3 x 112 bytes)


def _fake_prove(kws):
    import xfgstark
    out = []
    for i, kw in enumerate(kws):
        pub, nf, cm = xfgstark.air_consts(**kw)
        b = struct.pack("<14Q", *pub, nf, cm)
        out.append(b * (1 + (pub[2] % 3)))  # variable-length "proofs"
    return out


class _FakeRecordBatch:
    """a submitted batch writing into an exchange record like PendingBatch.record_ready: int64
    lengths, then one FAKE_CAP slot per proof; `fail` = index of a proof that fails (length 0), or
    "batch": the whole batch fails (xfg_batch_wait's status; every length zeroed)"""

    def __init__(self, kws, record, fail=None):
        self.kws, (self.addr, self.nbytes, self.owner), self.fail = kws, record, fail

    def record_ready(self):
        proofs = _fake_prove(self.kws)
        k = len(proofs)
        assert self.nbytes >= 8 * k + k * FAKE_CAP
        hdr = (C.c_int64 * k).from_address(self.addr)
        for i, p in enumerate(proofs):
            hdr[i] = 0 if self.fail in (i, "batch") else len(p)
            C.memmove(self.addr + 8 * k + i * FAKE_CAP, p, len(p))
        if self.fail == "batch":
            raise RuntimeError("batch failed")
        if self.fail is not None:  # as PendingBatch.record_ready: length zeroed, then raise
            raise RuntimeError(f"proof {self.fail} failed")


def _worker(rank, world, port, per, ret, steps=3, depth=2, lookahead=4, fail=None):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "xfg-stark_amd"), root):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import bench
    import synthetic
    dist.init_process_group("gloo", rank=rank, world_size=world)
    batches = [[synthetic.burn_inputs(100 * k + i) for i in range(per * world)] if rank == 0 else None
               for k in range(steps)]
    packed = [torch.from_numpy(bench.pack_inputs(b)).view(world, per, bench.REC) if rank == 0 else None
              for b in batches]
    seen = []

    def submit(kws, record):
        seen.append(len(kws))
        return _FakeRecordBatch(kws, record, fail if rank == world - 1 else None)

    ex = bench.Exchange(rank, world, per, FAKE_CAP, torch.device("cpu"), dist, send_slots=depth + 3,
                        lookahead=lookahead)
    try:
        out = bench.pipelined_steps(submit, None, batches, depth, ex, packed)
    except RuntimeError as e:
        ret.put((rank, "error", str(e)))
        out = "raised"
    assert seen == [per] * steps
    if rank == 0:
        if out != "raised":
            ret.put((rank, "ok", [bytes(x) for x in out]))  # rank 0 holds zero-copy views into the ring
    else:
        assert out in (None, "raised")
    ex.close()
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(world, per, expect=1, **kw):
    """run the ranks; the first `expect` (rank, kind, payload) results, by rank"""
    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per, ret), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(ret.get(timeout=120) for _ in range(expect))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out[0][1:] if expect == 1 else out


@pytest.mark.parametrize("world,per,steps,depth,lookahead", [
    (2, 3, 1, 1, 4),   # one synchronous step
    (2, 1, 3, 2, 1),   # scatter only one step ahead
    (2, 2, 3, 2, 4),   # lookahead past the window
    (2, 2, 5, 3, 2),
    (4, 2, 4, 2, 3),   # four ranks
    (4, 1, 9, 2, 3),   # more steps than send records and receive slots
    (8, 2, 7, 2, 3),   # eight ranks, as on the driver's 8-GPU node
])
def test_exchange_gloo(world, per, steps, depth, lookahead):
    import synthetic
    kind, out = _run(world, per, steps=steps, depth=depth, lookahead=lookahead)
    assert kind == "ok"
    base = 100 * (steps - 1)  # the last step's inputs, in rank order
    want = _fake_prove([synthetic.burn_inputs(base + i) for i in range(per * world)])
    assert out == want


def test_exchange_failed_proof_raises_on_rank0():
    """a proof that failed on another rank (length 0 in its record) must not be read as a proof on
    rank 0, and the failing rank raises too -- after the window's collectives, so that no rank is
    left waiting in a gather (every step here fails on rank 1)"""
    (r0, k0, m0), (r1, k1, m1) = _run(2, 2, expect=2, steps=3, depth=2, fail=1)
    assert (r0, k0, r1, k1) == (0, "error", 1, "error")
    assert "rank 1 proof 1" in m0 and m1 == "proof 1 failed"


def test_exchange_batch_failure_raises_on_rank0():
    """a whole batch that failed on another rank (every length zeroed by record_ready) is rejected
    on rank 0 at its first proof, and the failing rank raises its own error"""
    (r0, k0, m0), (r1, k1, m1) = _run(2, 2, expect=2, steps=2, depth=2, fail="batch")
    assert (r0, k0, r1, k1) == (0, "error", 1, "error")
    assert "rank 1 proof 0" in m0 and m1 == "batch failed"


def test_record_ready_zeroes_lengths_on_batch_failure():
    """PendingBatch.record_ready itself: when xfg_batch_wait fails for the whole batch (every
    per-proof status 0, header words still at the capacity the submission wrote), every length in
    the caller's record is zeroed before it raises; a per-proof failure zeroes only that proof"""
    import xfgstark

    class _P:
        _free = []

        def _err(self, st):
            return xfgstark.XfgStarkError(st, "batch failed")

    for wst, sts, want in ((7, [0, 0, 0], [0, 0, 0]), (0, [0, 5, 0], [4096, 0, 4096])):
        lens = (C.c_int64 * 3)(4096, 4096, 4096)
        st_arr = (C.c_int * 3)(*sts)
        pb = xfgstark.PendingBatch(_P(), 0, None, 0, 4096, None, lens, st_arr, record=True)
        pb._wst = wst  # as if xfg_batch_wait had returned it
        with pytest.raises(xfgstark.XfgStarkError):
            pb.record_ready()
        assert list(lens) == want
        with pytest.raises(xfgstark.XfgStarkError):  # no views of a failed batch
            pb.record_views()
    # a successful batch: zero-copy views of each proof's used bytes in the caller's record
    cap, k = 64, 3
    rec = (C.c_uint8 * (8 * k + cap * k))()
    lens = (C.c_int64 * k).from_buffer(rec)
    body = [bytes([7 + i]) * (10 + 20 * i) for i in range(k)]
    for i, b in enumerate(body):
        lens[i] = len(b)
        C.memmove(C.addressof(rec) + 8 * k + i * cap, b, len(b))
    pb = xfgstark.PendingBatch(_P(), 0, None, C.addressof(rec) + 8 * k, cap, None, lens, (C.c_int * k)(), record=True,
                               owner=rec)
    pb._wst = 0
    pb.record_ready()
    views = pb.record_views()
    assert [bytes(v) for v in views] == body
    rec[8 * k] = 99  # views, not copies
    assert views[0][0] == 99


def test_pack_unpack_roundtrip():
    import bench
    import synthetic
    kws = [synthetic.burn_inputs(i) for i in range(5)] + [synthetic.REFERENCE_PACKAGE]
    assert bench.unpack_inputs(bench.pack_inputs(kws)) == kws


class _Work:
    def wait(self):
        pass

    def is_completed(self):
        return True


class _LoopbackDist:
    """two "ranks" in one process, seen from rank 0: rank 1's record is handed to rank 0's gather
    and rank 0's scatter keeps chunk 0 (exercises the device-tensor branch of bench.Exchange --
    side stream, pinned records, events -- on one GPU)"""

    def __init__(self, other):
        self.other = other

    def scatter(self, t, chunks, src=0, group=None, async_op=False):
        t.copy_(chunks[0])
        return _Work()

    def gather(self, t, got, dst=0, group=None, async_op=False):
        got[0].copy_(t)
        got[1].copy_(self.other.to(t.device))
        return _Work()


def _read_dump(path):
    data, out, off = open(path, "rb").read(), [], 0
    while off < len(data):
        ln = int.from_bytes(data[off:off + 4], "little")
        out.append(data[off + 4:off + 4 + ln])
        off += 4 + ln
    return out


@pytest.mark.gpu
def test_bench_two_ranks_real_prover(tmp_path):
    """configs[3]'s sharded path with real proofs: bench.py under torch.distributed.run with TWO ranks
    sharing the one GPU (XFG_DIST_BACKEND=gloo: host-side scatter / gather tensors; RCCL cannot run
    two ranks on one device), 8 proofs per rank per step, 2^10-step traces. Rank 0 verifies every
    gathered proof of the last step against its statement on the GPU and (--dist) checks them byte
    for byte against a direct prove_batch of the same 16 inputs in order; here the dumped proofs are
    checked against the oracle: two of them byte for byte, all 16 through the oracle verifier.
    Started as a child process before this test process touches the GPU (the first GPU test of the
    session). Reference batch pattern: src/burn_mint_verifier.rs:326-338."""
    import json
    import subprocess
    import sys
    import oracle_lib as O
    import synthetic
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dump = tmp_path / "proofs.bin"
    per, world, steps, warmup, n = 8, 2, 2, 1, 1024
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(world), "--steps", str(steps), "--warmup", str(warmup), "--per-gpu", str(per),
           "--log-n", "10", "--depth", "2", "--no-cpu-baseline", "--no-config5", "--dist",
           "--dump-proofs", str(dump)]
    env = dict(os.environ, XFG_DIST_BACKEND="gloo")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world and line["verified"] == per * world
    got = _read_dump(dump)
    assert len(got) == per * world
    last = [synthetic.burn_inputs((warmup + steps - 1) * per * world + i) for i in range(per * world)]
    for i, kw in enumerate(last):
        st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"],
                                    kw["recipient_address"], kw["secret"])
        assert st == 0 and O.verify(air, got[i], O.options()) == 0, i
        if i in (0, per):  # the first proof of each rank's shard
            st, want = O.prove(air, n, O.options())
            assert st == 0 and got[i] == want, i


@pytest.mark.gpu
def test_exchange_device_branch():
    import sys
    import numpy as np
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    import synthetic
    per, cap, dev = 3, 400, torch.device("cuda", 0)
    kws = [synthetic.burn_inputs(i) for i in range(2 * per)]
    theirs = [bytes([50 + i]) * (300 - 11 * i) for i in range(per)]
    pay = np.zeros(8 * per + per * cap, dtype=np.uint8)  # rank 1's record: lengths, fixed slots
    pay[:8 * per] = np.array([len(p) for p in theirs], dtype=np.int64).view(np.uint8)
    for i, p in enumerate(theirs):
        pay[8 * per + i * cap:8 * per + i * cap + len(p)] = np.frombuffer(p, dtype=np.uint8)
    ex = bench.Exchange(0, 2, per, cap, dev, _LoopbackDist(torch.from_numpy(pay)), send_slots=3, lookahead=2)
    packed = [torch.from_numpy(bench.pack_inputs(kws)).to(dev).view(2, per, bench.REC)] * 3
    ex.start_inputs(packed, 3)
    for step in range(3):
        assert ex.inputs(step) == kws[:per]  # rank 0's shard of each step
        s, addr, nbytes, _ = ex.claim()
        assert nbytes == len(pay)
        k = len(kws[:per])
        mine = _fake_prove(kws[:per])
        hdr = (C.c_int64 * k).from_address(addr)
        for i, p in enumerate(mine):
            hdr[i] = len(p)
            C.memmove(addr + 8 * k + i * cap, p, len(p))
        out = ex.gather(s).proofs()
        assert [bytes(x) for x in out] == mine + theirs
    ex.drain()
    ex.close()


@pytest.mark.gpu
def test_bench_rccl_collectives_one_rank():
    """bench.py's exchange step over RCCL itself (backend nccl: device tensors, one scatter of packed
    inputs per step, gather of fixed-size proof records, pinned D2H), one rank on the
    one-GPU box through torch.distributed.run -- the path the driver's multi-GPU runs take. bench.py
    --dist checks that the gathered proofs equal a direct prove_batch of the same inputs."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--per-gpu", "8", "--depth", "2",
           "--no-cpu-baseline", "--no-config5", "--dist"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["value"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_config3_eight_ranks_real_prover(tmp_path):
    """BASELINE configs[3] at its workload: 512 burn proofs per step (2^16-step traces, blowup 8, the
    reference options) sharded over EIGHT bench.py ranks under torch.distributed.run, 64 proofs per
    rank, all sharing the one GPU (XFG_DIST_BACKEND=gloo: RCCL cannot put two ranks on one device;
    the driver's 8-GPU node runs the same code over nccl). Rank 0 GPU-verifies all 512 gathered
    proofs of the last step against the statements of the inputs in rank order and (--dist) compares
    them byte for byte with a direct prove_batch of the same 512 inputs; here the first proof of
    every rank's shard must equal the oracle's bytes and all 512 must pass the oracle verifier.
    Reference batch pattern: src/burn_mint_verifier.rs:326-338, harness src/benchmarks/mod.rs:301-342."""
    import json
    import subprocess
    import sys
    from concurrent.futures import ThreadPoolExecutor
    import oracle_lib as O
    import synthetic
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dump = tmp_path / "proofs.bin"
    per, world, steps, warmup, n = 64, 8, 2, 1, 1 << 16
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", str(world), "--steps", str(steps), "--warmup", str(warmup), "--per-gpu", str(per),
           "--log-n", "16", "--depth", "2", "--no-cpu-baseline", "--no-config5", "--dist",
           "--dump-proofs", str(dump)]
    # 3 lanes per rank: 8 contexts share the card's memory and hardware queues
    env = dict(os.environ, XFG_DIST_BACKEND="gloo", XFG_LANES="3", OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=840, cwd=root, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world and line["config"]["proofs_per_step"] == 512
    assert line["verified"] == per * world
    got = _read_dump(dump)
    assert len(got) == per * world
    last = [synthetic.burn_inputs((warmup + steps - 1) * per * world + i) for i in range(per * world)]
    airs = []
    for kw in last:
        st, air = O.air_from_inputs(kw["burn_amount"], kw["mint_amount"], kw["tx_prefix_hash"],
                                    kw["recipient_address"], kw["secret"])
        assert st == 0
        airs.append(air)
    opts = O.options()
    with ThreadPoolExecutor(16) as pool:
        verdicts = list(pool.map(lambda i: O.verify(airs[i], got[i], opts), range(len(got))))
        firsts = list(pool.map(lambda q: O.prove(airs[q * per], n, opts), range(world)))
    assert verdicts == [0] * len(got)
    for q, (st, want) in enumerate(firsts):  # the first proof of each rank's shard
        assert st == 0 and got[q * per] == want, q


def test_bench_launch_limit_kills_the_ranks(monkeypatch):
    """a rank that hangs (here: a child that prints, then sleeps) is terminated with its whole
    process group once the wall-clock limit passes, and launch_ranks returns non-zero"""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    real, procs = subprocess.Popen, []

    def hang(cmd, **kw):
        p = real([sys.executable, "-c", "import time; print('rank up', flush=True); time.sleep(120)"], **kw)
        procs.append(p)
        return p

    monkeypatch.setattr(subprocess, "Popen", hang)
    t = time.time()
    assert bench.launch_ranks(2, ["--steps", "1"], limit_s=2) != 0
    assert time.time() - t < 30 and procs[0].poll() is not None


def test_rank_cpu_slices():
    """bench.py pins each rank of a node to a disjoint slice of the CPUs it may use (the driver's
    8-GPU node: 8 ranks) and sizes the host pool to the slice"""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    cpus = set(range(16, 144))  # 128 CPUs, not starting at 0
    sl = [bench.rank_cpus(r, 8, cpus) for r in range(8)]
    assert all(len(x) == 16 for x in sl) and len(set().union(*map(set, sl))) == 128
    assert sl[0][0] == 16 and sl[7][-1] == 143
    assert bench.rank_cpus(0, 1, cpus) == sorted(cpus)           # one rank: everything
    assert bench.rank_cpus(3, 8, {0, 1, 2}) == [0, 1, 2]          # fewer CPUs than ranks: no split
    assert [bench.rank_cpus(r, 3, range(8)) for r in range(3)] == [[0, 1], [2, 3], [4, 5]]
    assert [bench.host_threads_for(k) for k in (1, 2, 4, 16, 32)] == [2, 2, 2, 8, 8]


def _fake_sysfs(root, gpus):
    """a KFD topology with one CPU node and `gpus` = [(pci bus, local_cpulist)] GPU nodes"""
    nodes = root / "class" / "kfd" / "kfd" / "topology" / "nodes"
    (nodes / "0").mkdir(parents=True)
    (nodes / "0" / "properties").write_text("cpu_cores_count 128\nsimd_count 0\n")
    for i, (bus, cl) in enumerate(gpus):
        d = nodes / str(i + 1)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        dev = root / "bus" / "pci" / "devices" / f"0000:{bus:02x}:00.0"
        dev.mkdir(parents=True)
        (dev / "local_cpulist").write_text(cl + "\n")


def test_rank_cpu_slices_numa(tmp_path):
    """on a two-socket node (GPUs 0-3 next to CPUs 0-63,128-191, GPUs 4-7 next to 64-127,192-255),
    every rank's slice lies in its own GPU's local set, the slices are disjoint, and each takes a
    quarter of its socket; *_VISIBLE_DEVICES lists are followed; a missing topology or a non-index
    visibility list falls back to the contiguous split"""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    s0, s1 = "0-63,128-191", "64-127,192-255"
    _fake_sysfs(tmp_path, [(0x10 + 0x10 * g, s0 if g < 4 else s1) for g in range(8)])
    assert bench.parse_cpulist(s0) == set(range(64)) | set(range(128, 192))
    env = {}
    local = [bench.gpu_local_cpus(r, sysfs=str(tmp_path), env=env) for r in range(8)]
    assert local[0] == bench.parse_cpulist(s0) and local[7] == bench.parse_cpulist(s1)
    sl = [bench.rank_cpus_local(r, 8, range(256), local) for r in range(8)]
    assert all(len(x) == 32 and set(x) <= local[r] for r, x in enumerate(sl))
    assert len(set().union(*map(set, sl))) == 256
    # the contiguous split would have put ranks 2, 3 on the other socket
    assert not set(bench.rank_cpus(2, 8, range(256))) <= local[2]
    # visibility lists index into the previous list: ROCr's, then HIP's
    vis = {"ROCR_VISIBLE_DEVICES": "6,2,5", "HIP_VISIBLE_DEVICES": "2,1"}
    assert [bench.gpu_local_cpus(r, sysfs=str(tmp_path), env=vis) for r in range(2)] == [local[5], local[2]]
    assert bench.gpu_local_cpus(0, sysfs=str(tmp_path), env={"HIP_VISIBLE_DEVICES": "GPU-1234"}) is None
    assert bench.gpu_local_cpus(0, sysfs=str(tmp_path), env={"ROCR_VISIBLE_DEVICES": "9"}) is None
    assert bench.gpu_local_cpus(0, sysfs=str(tmp_path / "none"), env=env) is None
    assert bench.rank_cpus_local(1, 2, range(8), [None, {0, 1}]) == bench.rank_cpus(1, 2, range(8))
    # a node whose other cards this process may not open: only the readable GPU node counts
    part = tmp_path / "part"
    _fake_sysfs(part, [(0x10, s0), (0x20, s1)])
    prop = part / "class" / "kfd" / "kfd" / "topology" / "nodes" / "1" / "properties"
    prop.chmod(0)
    if os.geteuid() != 0:  # root reads mode-0 files anyway
        assert bench.gpu_local_cpus(0, sysfs=str(part), env=env) == bench.parse_cpulist(s1)
    # ranks sharing one GPU (the one-GPU rehearsals): its local set split between them
    one = tmp_path / "one"
    _fake_sysfs(one, [(0x10, "0-15")])
    loc = [bench.gpu_local_cpus(r, sysfs=str(one), env=env) for r in range(2)]
    assert [bench.rank_cpus_local(r, 2, range(64), loc) for r in range(2)] == [list(range(8)), list(range(8, 16))]


def test_bench_gpus_mismatch_fails_loudly():
    """under a launcher, --gpus must equal WORLD_SIZE: a mismatch exits non-zero before any GPU work
    instead of printing a line for a different N"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8"], capture_output=True,
                       text=True, timeout=60, cwd=root, env=env)
    assert r.returncode != 0 and "--gpus 8 but the launcher started WORLD_SIZE=2" in r.stderr


def test_bench_launch_command(monkeypatch):
    """bench.py --gpus N without WORLD_SIZE starts torch.distributed.run with N ranks on 127.0.0.1 as a
    child, passes its own arguments through, relays JSON lines to stdout and returns the child's code"""
    import io
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    seen = {}

    class FakePopen:
        def __init__(self, cmd, **kw):
            seen["cmd"] = cmd
            self.stdout = io.StringIO('torchrun chatter\n{"metric": "m", "n_gpus": 4}\n')

        def wait(self, timeout=None):
            return 3

        def poll(self):
            return 3

    monkeypatch.setattr(subprocess, "Popen", FakePopen)
    out, err = io.StringIO(), io.StringIO()
    monkeypatch.setattr(sys, "stdout", out)
    monkeypatch.setattr(sys, "stderr", err)
    assert bench.launch_ranks(4, ["--gpus", "4", "--steps", "2"]) == 3
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"] and cmd[-5].endswith("bench.py")
    assert out.getvalue() == '{"metric": "m", "n_gpus": 4}\n' and "torchrun chatter" in err.getvalue()
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == 4 and bench.check_world(1, {}) == 1


@pytest.mark.gpu
def test_bench_gpus_two_without_launcher():
    """the driver's plain form `bench.py --gpus 2` (no torch.distributed.run in the command) runs two
    ranks by itself: here sharing the one GPU over gloo, 8 proofs each, all 16 of the last step
    gathered and GPU-verified on rank 0"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--per-gpu", "8", "--log-n", "10",
           "--steps", "2", "--warmup", "1", "--depth", "2", "--no-cpu-baseline", "--no-config5"]
    env = dict(os.environ, XFG_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=root, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.strip().splitlines() if x.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["verified"] == 16 and line["config"]["proofs_per_step"] == 16
    ex, load = line["exchange"], line["host_load"]
    assert ex["world"] == 2 and [r[0] for r in ex["ranks"]] == [0, 1]
    assert [r["rank"] for r in load] == [0, 1] and all(r["cpu_s_per_step"] > 0 for r in load)
    if len(os.sched_getaffinity(0)) >= 2:  # two disjoint affinity slices
        assert load[0]["cpu_first"] + load[0]["cpus"] <= load[1]["cpu_first"]


@pytest.mark.gpu
def test_bench_emulated_eight_rank_gather():
    """rank 0's N = 8 exchange load on one GPU over RCCL (--dist --emulate-ranks 8): eight real-size
    records received per step, the D2H of all eight, and every received copy equal to the proofs"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--per-gpu", "8", "--depth", "2", "--log-n", "10",
           "--no-cpu-baseline", "--no-config5", "--dist", "--emulate-ranks", "8"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["exchange"]["records_received_per_step"] == 8 and line["verified"] == 8


def test_bench_roofline_records():
    """bench.py's roofline fields read the newest committed records: the trace-LDE PMC record of the
    64-proof 2^16 launch set (traffic, lane instructions per output) and the whole-proof VALU ledger
    with its instruction-mix ceiling; SURVEY 8(d)'s per-proof algorithmic bytes at configs[2]"""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    assert bench.whole_proof_bytes(1 << 16, 8) == 221_246_464
    rec, src = bench.pmc_record(64, 1 << 16, 8)
    assert rec and src.startswith("profiles/r") and rec["traffic_bytes"] > rec["algorithmic_bytes"]
    v = bench.valu_roofline(rec, 1.4, 7 * 64 * (1 << 16) * 8)
    assert 150 < v["lane_instr_per_output"] < 200 and 0 < v["frac"] < 1.2
    w = bench.whole_proof_valu(14000.0, 1 << 16, 1)
    assert w and w["ceiling_T_lane_instr_s"] > 36 and 0 < w["frac"] < 1 and w["source"].endswith("valu_per_proof.json")
    assert bench.whole_proof_valu(14000.0, 1 << 20, 1) is None  # the ledger is for configs[2] only
    assert bench.whole_proof_valu(28000.0, 1 << 16, 2)["ceiling_T_lane_instr_s"] == 2 * w["ceiling_T_lane_instr_s"]
