"""ctypes binding of the CPU parity oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package.
"""
import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")


class Options(C.Structure):
    _fields_ = [("num_queries", C.c_uint32), ("blowup", C.c_uint32), ("grinding", C.c_uint32),
                ("field_extension", C.c_uint32), ("fri_folding", C.c_uint32), ("fri_rem_max_deg", C.c_uint32)]


class Air(C.Structure):
    _fields_ = [("pub", C.c_uint64 * 12), ("secret", C.c_uint64), ("nullifier", C.c_uint64),
                ("commitment", C.c_uint64)]


class Debug(C.Structure):
    _fields_ = [("trace_root", C.c_uint8 * 32), ("constraint_root", C.c_uint8 * 32),
                ("fri_roots", (C.c_uint8 * 32) * 16), ("num_fri_layers", C.c_uint32), ("z", C.c_uint64),
                ("ood", C.c_uint64 * 15), ("pow_nonce", C.c_uint64), ("num_unique_queries", C.c_uint32),
                ("positions", C.c_uint64 * 256)]


REFERENCE_OPTIONS = dict(num_queries=42, blowup=8, grinding=4, field_extension=1, fri_folding=8, fri_rem_max_deg=31)

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        u8p, u64p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)
        L.orc_blake3_bytes.argtypes = [C.c_char_p, C.c_size_t, u8p]
        L.orc_keccak256_bytes.argtypes = [C.c_char_p, C.c_size_t, u8p]
        L.orc_sha3_256_bytes.argtypes = [C.c_char_p, C.c_size_t, u8p]
        L.orc_field_mul.restype = C.c_uint64
        L.orc_field_mul.argtypes = [C.c_uint64, C.c_uint64]
        L.orc_field_root.restype = C.c_uint64
        L.orc_field_root.argtypes = [C.c_uint32]
        L.orc_burn_air_from_inputs.argtypes = [C.c_uint64, C.c_uint64, C.c_char_p, C.c_char_p, C.c_size_t,
                                               C.c_char_p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_uint32,
                                               C.POINTER(Air)]
        L.orc_air_constants.argtypes = [u64p, C.c_uint64, u64p, u8p, u64p]
        L.orc_build_trace.argtypes = [C.POINTER(Air), C.c_uint64, u64p]
        L.orc_prove.argtypes = [C.POINTER(Air), u64p, C.c_uint64, C.POINTER(Options), C.c_int, u8p,
                                C.POINTER(C.c_size_t), C.POINTER(Debug)]
        L.orc_prove_batch.argtypes = [C.POINTER(Air), C.c_uint32, C.c_uint64, C.POINTER(Options), C.c_int, C.c_int,
                                      C.POINTER(C.c_size_t), C.POINTER(C.c_int), C.POINTER(C.c_double)]
        L.orc_proof_size_bound.restype = C.c_size_t
        L.orc_proof_size_bound.argtypes = [C.c_uint64, C.POINTER(Options)]
        L.orc_verify.argtypes = [C.POINTER(Air), C.c_char_p, C.c_size_t, C.POINTER(Options)]
        L.orc_eval_transition.argtypes = [C.POINTER(Air), u64p, u64p, u64p]
        L.orc_interpolate.argtypes = [u64p, C.c_uint64, C.c_uint64]
        L.orc_evaluate_lde.argtypes = [u64p, C.c_uint64, C.c_uint64, C.c_uint64, u64p]
        _lib = L
    return _lib


def blake3(data: bytes) -> bytes:
    out = (C.c_uint8 * 32)()
    lib().orc_blake3_bytes(data, len(data), out)
    return bytes(out)


def keccak256(data: bytes) -> bytes:
    out = (C.c_uint8 * 32)()
    lib().orc_keccak256_bytes(data, len(data), out)
    return bytes(out)


def sha3_256(data: bytes) -> bytes:
    out = (C.c_uint8 * 32)()
    lib().orc_sha3_256_bytes(data, len(data), out)
    return bytes(out)


def options(**kw):
    d = dict(REFERENCE_OPTIONS)
    d.update(kw)
    return Options(**d)


def air_from_inputs(burn, mint, tx_hash: bytes, recipient: bytes, secret: bytes, network_id=1,
                    target_chain_id=42161, commitment_version=1):
    a = Air()
    st = lib().orc_burn_air_from_inputs(burn, mint, tx_hash, recipient, len(recipient), secret, len(secret),
                                        network_id, target_chain_id, commitment_version, C.byref(a))
    return st, a


def build_trace(air, n):
    buf = (C.c_uint64 * (7 * n))()
    lib().orc_build_trace(C.byref(air), n, buf)
    return buf


def prove(air, n, opts, trace=None, faithful=False, debug=False):
    if trace is None:
        trace = build_trace(air, n)
    cap = lib().orc_proof_size_bound(n, C.byref(opts))
    out = (C.c_uint8 * cap)()
    ln = C.c_size_t(cap)
    dbg = Debug() if debug else None
    st = lib().orc_prove(C.byref(air), trace, n, C.byref(opts), 1 if faithful else 0, out, C.byref(ln),
                         C.byref(dbg) if dbg is not None else None)
    proof = bytes(out[:ln.value]) if st == 0 else None
    return (st, proof, dbg) if debug else (st, proof)


STAGES = ("trace_lde", "trace_commit", "constraint_eval", "composition", "ood_deep", "fri", "grinding_queries",
          "serialize")


def prove_batch(airs, n, opts, faithful=False, threads=0):
    """orc_prove_batch: len(airs) proofs over `threads` OpenMP threads (0 = OpenMP default).
    -> (threads used, [proof len], [status], {stage: summed CPU ms})"""
    k = len(airs)
    arr = (Air * k)(*airs)
    lens = (C.c_size_t * k)()
    sts = (C.c_int * k)()
    ms = (C.c_double * len(STAGES))()
    used = lib().orc_prove_batch(arr, k, n, C.byref(opts), 1 if faithful else 0, threads, lens, sts, ms)
    return used, list(lens), list(sts), dict(zip(STAGES, ms))


def verify(air, proof: bytes, opts) -> int:
    return lib().orc_verify(C.byref(air), proof, len(proof), C.byref(opts))


def eval_transition(air, cur, nxt):
    r = (C.c_uint64 * 7)()
    lib().orc_eval_transition(C.byref(air), (C.c_uint64 * 7)(*cur), (C.c_uint64 * 7)(*nxt), r)
    return list(r)


def interpolate(vals, offset=1):
    n = len(vals)
    buf = (C.c_uint64 * n)(*vals)
    lib().orc_interpolate(buf, n, offset)
    return list(buf)


def evaluate_lde(coef, blowup, offset=7):
    n = len(coef)
    cb = (C.c_uint64 * n)(*coef)
    out = (C.c_uint64 * (n * blowup))()
    lib().orc_evaluate_lde(cb, n, blowup, offset, out)
    return list(out)


def evaluate_lde_np(coef, blowup, offset=7):
    """evaluate_lde over numpy uint64 arrays (no Python-int lists: for the 2^20+ parity cases)"""
    import numpy as np
    cb = np.ascontiguousarray(coef, dtype=np.uint64)
    out = np.zeros(cb.size * blowup, dtype=np.uint64)
    lib().orc_evaluate_lde(cb.ctypes.data_as(C.POINTER(C.c_uint64)), cb.size, blowup, offset,
                           out.ctypes.data_as(C.POINTER(C.c_uint64)))
    return out


def interpolate_np(vals, offset=1):
    import numpy as np
    buf = np.array(vals, dtype=np.uint64, copy=True)
    lib().orc_interpolate(buf.ctypes.data_as(C.POINTER(C.c_uint64)), buf.size, offset)
    return buf
