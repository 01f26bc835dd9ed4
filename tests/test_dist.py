"""Multi-GPU path on CPU: bench.sharded_step over torch.distributed gloo with world_size 2.

Rank 0 scatters packed burn inputs, every rank "proves" its shard (here: the product's host
marshalling, xfgstark.air_consts, serialised -- variable-length outputs), rank 0 gathers the
bytes. The result must equal proving the whole batch on one rank, in order (independent proofs
shard with no data-path collective besides the input scatter / output gather)."""
import os
import socket
import struct

import pytest
import torch.multiprocessing as mp


def _fake_prove(kws):
    import xfgstark
    out = []
    for i, kw in enumerate(kws):
        pub, nf, cm = xfgstark.air_consts(**kw)
        b = struct.pack("<14Q", *pub, nf, cm)
        out.append(b * (1 + (pub[2] % 3)))  # variable-length "proofs"
    return out


def _worker(rank, world, port, per, ret, mode="sync"):
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
    if mode == "sync":
        inputs = [synthetic.burn_inputs(i) for i in range(per * world)] if rank == 0 else None
        out = bench.sharded_step(_fake_prove, inputs, rank, world, per, torch.device("cpu"), dist)
    else:
        # bench.py's timed loop: 3 steps, submission depth 2, inputs pre-packed on rank 0
        batches = [[synthetic.burn_inputs(100 * k + i) for i in range(per * world)] if rank == 0 else None
                   for k in range(3)]
        packed = [torch.from_numpy(bench.pack_inputs(b)).view(world, per, bench.REC) if rank == 0 else None
                  for b in batches]
        seen = []

        def submit(kws):
            seen.append(len(kws))
            return _fake_prove(kws)

        depth = 3 if mode == "pipelined3" else 2
        out = bench.pipelined_steps(submit, lambda p: p, batches, rank, world, per, torch.device("cpu"), dist,
                                    packed, depth)
        assert seen == [per] * 3
    if rank == 0:
        ret.put([bytes(x) for x in out])  # rank 0 holds zero-copy views into the gathered buffer
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world,per,mode", [(2, 3, "sync"), (2, 1, "sync"), (2, 2, "pipelined"), (2, 2, "pipelined3")])
def test_sharded_step_gloo(world, per, mode):
    import synthetic
    ctx = mp.get_context("spawn")
    ret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per, ret, mode)) for r in range(world)]
    for p in procs:
        p.start()
    out = ret.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    base = 200 if mode.startswith("pipelined") else 0  # pipelined: the last of 3 steps
    want = _fake_prove([synthetic.burn_inputs(base + i) for i in range(per * world)])
    assert out == want


def test_pack_unpack_roundtrip():
    import bench
    import synthetic
    kws = [synthetic.burn_inputs(i) for i in range(5)] + [synthetic.REFERENCE_PACKAGE]
    assert bench.unpack_inputs(bench.pack_inputs(kws)) == kws


class _LoopbackDist:
    """two "ranks" in one process: rank 1's payload is handed to rank 0's gather (exercises the
    device-tensor branch of bench.gather_proofs on one GPU)"""
    class ReduceOp:
        MAX = "max"

    def __init__(self, other):
        self.other = other

    def all_reduce(self, t, op=None):
        t.copy_(torch_max(t, self.other["size"]))

    def gather(self, t, got, dst=0):
        got[0].copy_(t)
        got[1].copy_(self.other["payload"].to(t.device))


def torch_max(a, b):
    import torch
    return torch.maximum(a, b.to(a.device))


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
def test_gather_proofs_device_branch():
    import sys
    import numpy as np
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    per = 3
    mine = [bytes([i]) * (100 + 37 * i) for i in range(per)]
    theirs = [bytes([50 + i]) * (300 - 11 * i) for i in range(per)]
    # rank 1's payload as gather_proofs builds it, padded to the common size
    hdr = 8 * per
    size = max(hdr + sum(map(len, mine)), hdr + sum(map(len, theirs)))
    pay = np.zeros(size, dtype=np.uint8)
    pay[:hdr] = np.array([len(p) for p in theirs], dtype=np.int64).view(np.uint8)
    pay[hdr:hdr + sum(map(len, theirs))] = np.frombuffer(b"".join(theirs), dtype=np.uint8)
    other = {"size": torch.tensor([size], dtype=torch.int64), "payload": torch.from_numpy(pay)}
    out = bench.gather_proofs(mine, 0, 2, per, torch.device("cuda", 0), _LoopbackDist(other))
    assert [bytes(x) for x in out] == mine + theirs


@pytest.mark.gpu
def test_bench_rccl_collectives_one_rank():
    """bench.py's exchange step over RCCL itself (backend nccl: device tensors, scatter of packed
    inputs, length all-reduce, padded gather, pinned D2H of the gathered proofs), one rank on the
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
