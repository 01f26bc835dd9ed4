"""xfgstark -- Python mirror of the reference prover API over the MI355X C ABI (libxfgstark.so).

Mirrors reference src/burn_mint_prover.rs (XfgBurnMintProver::new / with_options /
prove_burn_mint / get_proof_size / security_parameter / proof_options) and the Winterfell
ProofOptions / StarkProof surface it returns. All proving runs in libxfgstark.so (HIP kernels
for gfx950); there is no CPU fallback: if the library is missing this module fails to import, and
without a GPU the prover constructor raises.
"""
import ctypes as C
import mmap
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
# XFG_LIB: an alternative build of the same library (same-box A/B of kernel variants)
LIB_PATH = os.environ.get("XFG_LIB") or os.path.join(_PKG, "libxfgstark.so")
HEADER_PATH = os.path.join(os.path.dirname(_PKG), "include", "xfg_stark.h")

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libxfgstark.so not built at {LIB_PATH}: run `make -C xfg-stark_amd` "
                      "(or __graft_entry__.build()); the prover has no CPU fallback")

_lib = C.CDLL(LIB_PATH)

STATUS = {0: "OK", 1: "INVALID_BURN_AMOUNT", 2: "MINT_MISMATCH", 3: "ZERO_TX_HASH", 4: "BAD_RECIPIENT_LEN",
          5: "SHORT_SECRET", 6: "PROVER_ERROR", 7: "DEVICE_ERROR", 8: "BUFFER_TOO_SMALL", 9: "INVALID_ARGUMENT",
          10: "VERIFY_FAILED"}


class _Options(C.Structure):
    _fields_ = [("num_queries", C.c_uint32), ("blowup_factor", C.c_uint32), ("grinding_factor", C.c_uint32),
                ("field_extension", C.c_uint32), ("fri_folding_factor", C.c_uint32),
                ("fri_remainder_max_degree", C.c_uint32)]


class _BurnInputs(C.Structure):
    _fields_ = [("burn_amount", C.c_uint64), ("mint_amount", C.c_uint64), ("tx_prefix_hash", C.c_uint8 * 32),
                ("recipient_address", C.c_char_p), ("recipient_len", C.c_size_t), ("secret", C.c_char_p),
                ("secret_len", C.c_size_t), ("network_id", C.c_uint32), ("target_chain_id", C.c_uint32),
                ("commitment_version", C.c_uint32)]


class _AirConsts(C.Structure):
    _fields_ = [("pub_inputs", C.c_uint64 * 12), ("nullifier", C.c_uint64), ("commitment", C.c_uint64)]


class _ProofInfo(C.Structure):
    _fields_ = [("trace_width", C.c_uint32), ("trace_length", C.c_uint64), ("options", _Options),
                ("num_unique_queries", C.c_uint32), ("num_fri_layers", C.c_uint32), ("remainder_len", C.c_uint32),
                ("pow_nonce", C.c_uint64), ("trace_root", C.c_uint8 * 32), ("constraint_root", C.c_uint8 * 32),
                ("ood_trace", C.c_uint64 * 14), ("ood_composition", C.c_uint64), ("size", C.c_size_t)]


_u64p = C.POINTER(C.c_uint64)
_u8p = C.POINTER(C.c_uint8)
_lib.xfg_ctx_create.restype = C.c_void_p
_lib.xfg_ctx_create.argtypes = [C.c_int]
_lib.xfg_ctx_destroy.argtypes = [C.c_void_p]
_lib.xfg_default_options.argtypes = [C.POINTER(_Options)]
_lib.xfg_last_error.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
_lib.xfg_proof_size_bound.restype = C.c_size_t
_lib.xfg_proof_size_bound.argtypes = [C.c_uint64, C.POINTER(_Options)]
_lib.xfg_prove_burn_mint.argtypes = [C.c_void_p, C.POINTER(_BurnInputs), C.c_uint64, C.POINTER(_Options), _u8p,
                                     C.POINTER(C.c_size_t)]
_lib.xfg_prove_trace.argtypes = [C.c_void_p, _u64p, C.c_uint32, C.c_uint64, C.POINTER(_AirConsts),
                                 C.POINTER(_Options), _u8p, C.POINTER(C.c_size_t)]
_lib.xfg_prove_batch.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(_BurnInputs), C.c_uint64, C.POINTER(_Options),
                                 C.POINTER(_u8p), C.POINTER(C.c_size_t), C.POINTER(C.c_int)]
_lib.xfg_prove_batch_submit.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(_BurnInputs), C.c_uint64,
                                         C.POINTER(_Options), C.POINTER(_u8p), C.POINTER(C.c_size_t),
                                         C.POINTER(C.c_int), C.POINTER(C.c_uint64)]
_lib.xfg_batch_wait.argtypes = [C.c_void_p, C.c_uint64]
_lib.xfg_proof_parse.argtypes = [_u8p, C.c_size_t, C.POINTER(_ProofInfo), C.c_char_p, C.c_size_t]
_lib.xfg_verify.argtypes = [_u8p, C.c_size_t, C.POINTER(_AirConsts), C.POINTER(_Options), C.c_char_p, C.c_size_t]
_lib.xfg_verify_batch.argtypes = [C.c_uint32, C.POINTER(_u8p), C.POINTER(C.c_size_t), C.POINTER(_AirConsts),
                                  C.POINTER(_Options), C.POINTER(C.c_int), C.c_uint32]
_lib.xfg_verify_batch_gpu.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(_u8p), C.POINTER(C.c_size_t),
                                      C.POINTER(_AirConsts), C.POINTER(_Options), C.POINTER(C.c_int)]
_lib.xfg_selftest_blake3.argtypes = [_u8p, C.c_size_t, _u8p]
_lib.xfg_prepare.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.POINTER(_Options)]
_lib.xfg_burn_air_consts.argtypes = [C.POINTER(_BurnInputs), C.POINTER(_AirConsts)]
_lib.xfg_set_timing.argtypes = [C.c_void_p, C.c_int]
_lib.xfg_stage_times.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_char_p), C.c_int]
_lib.xfg_bench_lde.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(C.c_double)]
_lib.xfg_lde_probe.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                               C.POINTER(C.c_uint64)]
_lib.xfg_debug_lde.argtypes = [C.c_void_p, _u64p, C.c_uint32, C.c_uint64, C.c_uint32, _u64p]
_lib.xfg_debug_ood_deep.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, _u64p, _u64p, _u64p, _u64p, _u64p, _u64p]
_lib.xfg_debug_interpolate.argtypes = [C.c_void_p, _u64p, C.c_uint32, C.c_uint64, C.c_int, _u64p]
if hasattr(_lib, "xfg_debug_field"):  # absent from builds older than the primitive self test (XFG_LIB A/B)
    _lib.xfg_debug_field.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, _u64p, _u64p, _u64p]
if hasattr(_lib, "xfg_debug_coin_draws"):  # absent from builds older than the device transcript
    _lib.xfg_debug_coin_draws.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.c_uint64, C.c_uint32, C.c_uint32,
                                          _u64p, _u64p, _u64p, _u64p, C.POINTER(C.c_int)]


class XfgStarkError(Exception):
    """XfgStarkError::CryptoError(String) (reference src/lib.rs:66-110); `.status` is the C-ABI code."""

    def __init__(self, status, message):
        super().__init__(message)
        self.status = status
        self.kind = STATUS.get(status, str(status))


class FieldExtension:
    NONE = 1
    QUADRATIC = 2
    CUBIC = 3


class ProofOptions:
    """winterfell::ProofOptions::new(num_queries, blowup_factor, grinding_factor, field_extension,
    fri_folding_factor, fri_remainder_max_degree) -- argument order of winter-air 0.8."""

    def __init__(self, num_queries, blowup_factor, grinding_factor, field_extension, fri_folding_factor,
                 fri_remainder_max_degree):
        self.num_queries = num_queries
        self.blowup_factor = blowup_factor
        self.grinding_factor = grinding_factor
        self.field_extension = field_extension
        self.fri_folding_factor = fri_folding_factor
        self.fri_remainder_max_degree = fri_remainder_max_degree

    @classmethod
    def reference(cls):
        """XfgBurnMintProver::new's ProofOptions::new(42, 8, 4, None, 8, 31) (src/burn_mint_prover.rs:28-35)."""
        o = _Options()
        _lib.xfg_default_options(C.byref(o))
        return cls(o.num_queries, o.blowup_factor, o.grinding_factor, o.field_extension, o.fri_folding_factor,
                   o.fri_remainder_max_degree)

    def _c(self):
        return _Options(self.num_queries, self.blowup_factor, self.grinding_factor, self.field_extension,
                        self.fri_folding_factor, self.fri_remainder_max_degree)

    def __repr__(self):
        return ("ProofOptions(num_queries={0.num_queries}, blowup_factor={0.blowup_factor}, grinding_factor="
                "{0.grinding_factor}, field_extension={0.field_extension}, fri_folding_factor="
                "{0.fri_folding_factor}, fri_remainder_max_degree={0.fri_remainder_max_degree})").format(self)


def _bytes_ptr(b):
    return C.cast(C.c_char_p(b), _u8p)


class StarkProof:
    """Serialized winterfell::StarkProof (to_bytes layout: DESIGN.md "Proof format").
    StarkProof.from_bytes parses and validates the structure (xfg_proof_parse); the parsed header is
    exposed as attributes (trace_length, options, num_unique_queries, pow_nonce, ...)."""

    def __init__(self, data: bytes):
        self._data = bytes(data)
        self._info = None

    @classmethod
    def from_bytes(cls, data: bytes):
        p = cls(data)
        p._parse()
        return p

    def _parse(self):
        if self._info is None:
            info, err = _ProofInfo(), C.create_string_buffer(256)
            st = _lib.xfg_proof_parse(_bytes_ptr(self._data), len(self._data), C.byref(info), err, 256)
            if st:
                raise XfgStarkError(st, err.value.decode())
            self._info = info
        return self._info

    def to_bytes(self) -> bytes:
        return self._data

    @property
    def trace_length(self):
        return self._parse().trace_length

    @property
    def options(self):
        o = self._parse().options
        return ProofOptions(o.num_queries, o.blowup_factor, o.grinding_factor, o.field_extension,
                            o.fri_folding_factor, o.fri_remainder_max_degree)

    @property
    def num_unique_queries(self):
        return self._parse().num_unique_queries

    @property
    def num_fri_layers(self):
        return self._parse().num_fri_layers

    @property
    def remainder_len(self):
        """FRI remainder coefficients (E elements)"""
        return self._parse().remainder_len

    @property
    def pow_nonce(self):
        return self._parse().pow_nonce

    @property
    def trace_root(self):
        return bytes(self._parse().trace_root)

    @property
    def constraint_root(self):
        return bytes(self._parse().constraint_root)

    @property
    def ood_frame(self):
        """([T_c(z)], [T_c(z g)], H(z))"""
        i = self._parse()
        return list(i.ood_trace[0::2]), list(i.ood_trace[1::2]), i.ood_composition

    def __len__(self):
        return len(self._data)

    def __eq__(self, other):
        return isinstance(other, StarkProof) and other._data == self._data


def _air_struct(air):
    pub, nullifier, commitment = air
    a = _AirConsts()
    a.pub_inputs = (C.c_uint64 * 12)(*pub)
    a.nullifier = nullifier
    a.commitment = commitment
    return a


class XfgBurnMintVerifier:
    """Mirror of the reference XfgBurnMintVerifier (src/burn_mint_verifier.rs:78-316) over
    xfg_verify. The statement of a proof is its AIR constants `air` = (public inputs[12], nullifier,
    commitment), as returned by air_consts(); acceptable options default to the reference's
    ProofOptions::new(42, 8, 4, None, 8, 31) (:95-110)."""

    def __init__(self, security_parameter=128, proof_options=None):
        self.security_parameter = security_parameter
        self.proof_options = proof_options or ProofOptions.reference()

    @classmethod
    def with_options(cls, security_parameter, proof_options):
        return cls(security_parameter, proof_options)

    def verify_with_details(self, proof, air):
        """-> (accepted, error text or None, proof size)"""
        data = proof.to_bytes() if isinstance(proof, StarkProof) else bytes(proof)
        a, o, err = _air_struct(air), self.proof_options._c(), C.create_string_buffer(256)
        st = _lib.xfg_verify(_bytes_ptr(data), len(data), C.byref(a), C.byref(o), err, 256)
        if st not in (0, 10):
            raise XfgStarkError(st, STATUS.get(st))
        return st == 0, (err.value.decode() or None), len(data)

    def verify_with_public_inputs(self, proof, air):
        return self.verify_with_details(proof, air)[0]

    def verify_burn_mint(self, proof, burn_amount, mint_amount, tx_prefix_hash, recipient_address, secret,
                         network_id=1, target_chain_id=42161, commitment_version=1):
        """statement rebuilt from the prover's inputs (the full 32-byte tx hash limbs included: the
        reference's zeroed limbs at :146-150 would reject every honest proof)"""
        air = air_consts(burn_amount, mint_amount, tx_prefix_hash, recipient_address, secret, network_id,
                         target_chain_id, commitment_version)
        return self.verify_with_public_inputs(proof, air)

    def batch_verify(self, proofs_and_airs, threads=0, gpu=None):
        """BatchBurnMintVerifier::verify_batch: list of (proof, air) -> list of bool. Host threads, or
        the GPU of `gpu` (an XfgBurnMintProver context) via xfg_verify_batch_gpu."""
        import numpy as np
        k = len(proofs_and_airs)
        if k == 0:
            return []
        datas = [(p.to_bytes() if isinstance(p, StarkProof) else bytes(p)) for p, _ in proofs_and_airs]
        # statements as one numpy array (per-item ctypes structs dominated large batches)
        ptrs = (_u8p * k)(*[_bytes_ptr(d) for d in datas])
        lens = (C.c_size_t * k)(*[len(d) for d in datas])
        air_np = np.array([list(a[0]) + [a[1], a[2]] for _, a in proofs_and_airs], dtype=np.uint64)
        airs = air_np.ctypes.data_as(C.POINTER(_AirConsts))
        res = (C.c_int * k)()
        o = self.proof_options._c()
        if gpu is not None:
            st = _lib.xfg_verify_batch_gpu(gpu._ctx, k, ptrs, lens, airs, C.byref(o), res)
            if st:
                raise gpu._err(st)
            return [r == 0 for r in res]
        st = _lib.xfg_verify_batch(k, ptrs, lens, airs, C.byref(o), res, threads)
        if st:
            raise XfgStarkError(st, STATUS.get(st))
        return [r == 0 for r in res]

    def verify_all(self, proofs_and_airs, threads=0):
        return all(self.batch_verify(proofs_and_airs, threads))


def blake3(data: bytes) -> bytes:
    """the library's host BLAKE3 (any length)"""
    out = (C.c_uint8 * 32)()
    _lib.xfg_selftest_blake3(_bytes_ptr(bytes(data)), len(data), out)
    return bytes(out)


def burn_inputs(burn_amount, mint_amount, tx_prefix_hash, recipient_address, secret, network_id=1,
                target_chain_id=42161, commitment_version=1):
    """pack prove_burn_mint arguments; keeps the referenced byte strings alive on the struct"""
    tx = bytes(tx_prefix_hash)
    if len(tx) != 32:
        raise XfgStarkError(9, "tx_prefix_hash must be 32 bytes ([u8; 32])")
    s = _BurnInputs()
    s.burn_amount = burn_amount
    s.mint_amount = mint_amount
    s.tx_prefix_hash = (C.c_uint8 * 32)(*tx)
    rcpt, sec = bytes(recipient_address), bytes(secret)
    s._keep = (rcpt, sec)
    s.recipient_address = rcpt
    s.recipient_len = len(rcpt)
    s.secret = sec
    s.secret_len = len(sec)
    s.network_id = network_id
    s.target_chain_id = target_chain_id
    s.commitment_version = commitment_version
    return s


def air_consts(burn_amount, mint_amount, tx_prefix_hash, recipient_address, secret, network_id=1,
               target_chain_id=42161, commitment_version=1):
    """(public inputs[12], nullifier, commitment) exactly as the prover derives them (host-side)."""
    s = burn_inputs(burn_amount, mint_amount, tx_prefix_hash, recipient_address, secret, network_id,
                    target_chain_id, commitment_version)
    a = _AirConsts()
    st = _lib.xfg_burn_air_consts(C.byref(s), C.byref(a))
    if st:
        raise XfgStarkError(st, STATUS[st])
    return list(a.pub_inputs), a.nullifier, a.commitment


def exported_symbols():
    return [name for name in dir(_lib)]


def _anon_map(size):
    """private anonymous mapping (the default mmap.mmap(-1, n) is MAP_SHARED: shmem pages, slower
    to fault and to write than the private pages malloc hands out)"""
    return mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)


def record_size(count, trace_length, options):
    """bytes of a fixed-size batch record (XfgBurnMintProver.submit_batch_record): `count` int64
    proof lengths, then `count` slots of xfg_proof_size_bound bytes, proof i at slot i"""
    o = options._c()
    return 8 * count + count * _lib.xfg_proof_size_bound(trace_length, C.byref(o))


class PendingBatch:
    """a submitted batch (XfgBurnMintProver.submit_batch); result() -> list of StarkProof | XfgStarkError.
    A batch is consumed once: by result() (which can be called again and returns the same list),
    by packed_into(), or -- for a batch written into a caller's record -- by record_ready()."""

    def __init__(self, prover, ticket, buf, base, cap, outs, lens, sts, record=False, owner=None):
        self._p, self._t, self._buf, self._base, self._cap = prover, ticket, buf, base, cap
        self._outs, self._lens, self._sts = outs, lens, sts
        self._record = record  # proofs live in the caller's record: no pooled buffer to release
        # the object owning the caller's record: kept alive while the workers may still write into
        # it (until the batch has been waited for, here or in __del__)
        self._owner = owner
        self._res = None
        self._consumed = None  # name of the call that consumed the batch, if not result()

    def _release(self):
        if self._buf is not None:
            self._p._free.append(self._buf)
            self._buf = None

    def wait(self):
        """block until every proof of the batch is done (idempotent); the batch's status code"""
        if not hasattr(self, "_wst"):
            self._wst = _lib.xfg_batch_wait(self._p._ctx, self._t)
        return self._wst

    def _check_unconsumed(self, what):
        if self._consumed:
            raise XfgStarkError(9, f"{what} after {self._consumed}(): the batch was already consumed")

    def result(self):
        if self._res is None:
            self._check_unconsumed("result")
            st = self.wait()
            if st:
                self._release()
                raise self._p._err(st)
            res = []
            for i in range(len(self._sts)):
                if self._sts[i]:
                    res.append(XfgStarkError(self._sts[i], STATUS.get(self._sts[i])))
                else:
                    res.append(StarkProof(C.string_at(self._base + i * self._cap, self._lens[i])))
            self._release()
            self._res = res
        return self._res

    def record_ready(self):
        """wait for a batch submitted with submit_batch_record; its record (lengths + fixed slots)
        is then complete in the caller's buffer. A failed proof raises (its length is zeroed in the
        record first, so a record that travels anyway cannot be read as a proof)."""
        if not self._record:
            raise XfgStarkError(9, "record_ready: the batch was not submitted into a record")
        self._check_unconsumed("record_ready")
        if self._res is not None:
            raise XfgStarkError(9, "record_ready after result()")
        self._consumed = "record_ready"
        st = self.wait()
        bad = [i for i in range(len(self._sts)) if self._sts[i]]
        # a batch-level failure leaves every status 0 and the header words at the capacity the
        # submission wrote: zero them all, so the record cannot be read as cap-byte proofs
        for i in (range(len(self._sts)) if st else bad):
            self._lens[i] = 0
        if st:
            raise self._p._err(st)
        if bad:
            raise XfgStarkError(self._sts[bad[0]], STATUS.get(self._sts[bad[0]]))
        return 8 * len(self._sts) + self._cap * len(self._sts)

    def record_views(self):
        """after record_ready(): every proof of the batch as a zero-copy memoryview into the caller's
        record (valid while the record is neither freed nor reused)"""
        if (self._consumed != "record_ready" or not hasattr(self, "_wst") or self._wst
                or any(self._sts[i] for i in range(len(self._sts)))):
            raise XfgStarkError(9, "record_views: call record_ready() first (and it must have succeeded)")
        return [memoryview((C.c_uint8 * self._cap).from_address(self._base + i * self._cap)).cast("B")[:self._lens[i]]
                for i in range(len(self._sts))]

    def packed_into(self, dst):
        """wait, then write the batch as one record into the uint8 numpy array `dst`: count int64
        lengths followed by the proof bytes back to back, straight from the workers' output buffer
        -- no per-proof bytes objects. Returns the record size. Any per-proof error raises."""
        import numpy as np
        if self._res is not None:
            raise XfgStarkError(9, "packed_into after result(): the batch's buffer was released")
        self._check_unconsumed("packed_into")
        self._consumed = "packed_into"
        st = self.wait()
        if st:
            self._release()
            raise self._p._err(st)
        k = len(self._sts)
        bad = [i for i in range(k) if self._sts[i]]
        lens = np.array([self._lens[i] for i in range(k)], dtype=np.int64)
        hdr = 8 * k
        need = hdr + int(lens.sum())
        if bad or need > dst.size:
            self._release()
            if bad:
                raise XfgStarkError(self._sts[bad[0]], STATUS.get(self._sts[bad[0]]))
            raise XfgStarkError(8, "packed_into: destination too small")
        dst[:hdr] = lens.view(np.uint8)
        base, off = dst.ctypes.data, hdr
        for i in range(k):
            C.memmove(base + off, self._base + i * self._cap, int(lens[i]))
            off += int(lens[i])
        self._release()
        return need

    def __del__(self, _finalizing=sys.is_finalizing):
        # the workers write into this batch's buffers: never release them before the batch is done;
        # a batch that was waited for but never consumed returns its buffer to the pool (the
        # finalizing check is bound at definition: module globals, `sys` included, are gone late in
        # interpreter teardown)
        if not _finalizing() and getattr(self._p, "_ctx", None):
            if self._res is None and not hasattr(self, "_wst"):
                _lib.xfg_batch_wait(self._p._ctx, self._t)
            self._release()


class XfgBurnMintProver:
    """reference XfgBurnMintProver (src/burn_mint_prover.rs:18-244) on one MI355X device."""

    def __init__(self, security_parameter=128, device=0, proof_options=None):
        self._security_parameter = security_parameter
        self._options = proof_options or ProofOptions.reference()
        self._ctx = _lib.xfg_ctx_create(device)
        if not self._ctx:
            raise XfgStarkError(7, f"no HIP device {device} available for libxfgstark (no CPU fallback)")

    @classmethod
    def new(cls, security_parameter=128, device=0):
        return cls(security_parameter, device)

    @classmethod
    def with_options(cls, security_parameter, proof_options, device=0):
        return cls(security_parameter, device, proof_options)

    def close(self):
        if getattr(self, "_ctx", None):
            _lib.xfg_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self, _finalizing=sys.is_finalizing):
        # at interpreter exit the module globals (`sys` and the HIP runtime included) may already be
        # gone -- hence the check bound at definition; process teardown releases the device buffers,
        # so only collect contexts dropped while running
        if not _finalizing():
            self.close()

    def _err(self, st):
        buf = C.create_string_buffer(1024)
        _lib.xfg_last_error(self._ctx, buf, 1024)
        return XfgStarkError(st, buf.value.decode() or STATUS.get(st, str(st)))

    def security_parameter(self):
        return self._security_parameter

    def proof_options(self):
        return self._options

    def get_proof_size(self, proof: StarkProof) -> int:
        return len(proof.to_bytes())

    def proof_size_bound(self, trace_length) -> int:
        """the largest proof this prover emits for `trace_length` under its options (xfg_proof_size_bound)"""
        o = self._options._c()
        return _lib.xfg_proof_size_bound(trace_length, C.byref(o))

    def prove_burn_mint(self, burn_amount, mint_amount, tx_prefix_hash, recipient_address, secret, network_id=1,
                        target_chain_id=42161, commitment_version=1, trace_length=64) -> StarkProof:
        s = burn_inputs(burn_amount, mint_amount, tx_prefix_hash, recipient_address, secret, network_id,
                        target_chain_id, commitment_version)
        o = self._options._c()
        cap = _lib.xfg_proof_size_bound(trace_length, C.byref(o))
        buf = C.create_string_buffer(cap)
        ln = C.c_size_t(cap)
        st = _lib.xfg_prove_burn_mint(self._ctx, C.byref(s), trace_length, C.byref(o), C.cast(buf, _u8p), C.byref(ln))
        if st:
            raise self._err(st)
        return StarkProof(C.string_at(buf, ln.value))

    def prove_trace(self, trace, pub_inputs, nullifier, commitment) -> StarkProof:
        """ExecutionTrace-level proving; trace = 7 columns of n canonical u64 (column-major)."""
        import numpy as np
        tr = np.ascontiguousarray(np.asarray(trace, dtype=np.uint64))
        width, n = tr.shape
        a = _AirConsts()
        a.pub_inputs = (C.c_uint64 * 12)(*pub_inputs)
        a.nullifier = nullifier
        a.commitment = commitment
        o = self._options._c()
        cap = _lib.xfg_proof_size_bound(n, C.byref(o))
        buf = C.create_string_buffer(cap)
        ln = C.c_size_t(cap)
        st = _lib.xfg_prove_trace(self._ctx, tr.ctypes.data_as(_u64p), width, n, C.byref(a), C.byref(o),
                                  C.cast(buf, _u8p), C.byref(ln))
        if st:
            raise self._err(st)
        return StarkProof(C.string_at(buf, ln.value))

    def prove_batch(self, inputs, trace_length=64):
        """list of dicts of prove_burn_mint kwargs -> list of StarkProof | XfgStarkError (per proof)."""
        return self.submit_batch(inputs, trace_length).result()

    def submit_batch(self, inputs, trace_length=64):
        """asynchronous prove_batch (xfg_prove_batch_submit): inputs are validated and marshalled
        now, proving runs on the context's lane workers; PendingBatch.result() waits. Submitting
        the next batch before collecting this one overlaps their host and device work."""
        k = len(inputs)
        arr = (_BurnInputs * k)()
        keep = []
        for i, kw in enumerate(inputs):
            s = burn_inputs(**kw)
            keep.append(s._keep)
            arr[i] = s
        o = self._options._c()
        cap = _lib.xfg_proof_size_bound(trace_length, C.byref(o))
        buf = self._take_buffer(cap * k)
        base = C.addressof(buf)
        outs = (_u8p * k)(*[C.cast(base + i * cap, _u8p) for i in range(k)])
        lens = (C.c_size_t * k)(*([cap] * k))
        sts = (C.c_int * k)()
        ticket = C.c_uint64(0)
        st = _lib.xfg_prove_batch_submit(self._ctx, k, arr, trace_length, C.byref(o), outs, lens, sts,
                                         C.byref(ticket))
        if st:
            self._free.append(buf)
            raise self._err(st)
        return PendingBatch(self, ticket.value, buf, base, cap, outs, lens, sts)

    def submit_batch_record(self, inputs, trace_length, addr, nbytes, owner=None):
        """submit_batch whose output is a caller-owned fixed-size record at host address `addr`
        (record_size bytes): the workers write proof i into slot i and its length into header word
        i, so the record can be handed to a collective (bench.py's exchange step) without packing.
        The record must stay untouched until PendingBatch.record_ready() returns; `owner` (the
        tensor, array or ctypes buffer holding it) is referenced by the PendingBatch so that the
        memory stays valid at least that long -- without it the caller must keep the record alive."""
        k = len(inputs)
        o = self._options._c()
        cap = _lib.xfg_proof_size_bound(trace_length, C.byref(o))
        if k == 0 or cap == 0 or nbytes < 8 * k + cap * k:
            raise XfgStarkError(9, f"submit_batch_record: record of {nbytes} B for {k} proofs of bound {cap} B")
        arr = (_BurnInputs * k)()
        keep = []
        for i, kw in enumerate(inputs):
            s = burn_inputs(**kw)
            keep.append(s._keep)
            arr[i] = s
        base = addr + 8 * k
        outs = (_u8p * k)(*[C.cast(base + i * cap, _u8p) for i in range(k)])
        lens = (C.c_size_t * k).from_address(addr)  # the record's header: capacity in, length out
        for i in range(k):
            lens[i] = cap
        sts = (C.c_int * k)()
        ticket = C.c_uint64(0)
        st = _lib.xfg_prove_batch_submit(self._ctx, k, arr, trace_length, C.byref(o), outs, lens, sts,
                                         C.byref(ticket))
        if st:
            raise self._err(st)
        return PendingBatch(self, ticket.value, None, base, cap, outs, lens, sts, record=True, owner=owner)

    def _take_buffer(self, size):
        # output buffers are recycled. A new one is an anonymous mapping, not create_string_buffer:
        # that zero-fills the whole bound (64 x 0.7 MB at n = 2^16) on the calling thread -- 11 ms
        # of page faults per batch, during which the next batch could not be submitted. The
        # mapping's pages are faulted in by the workers' proof copies instead, once.
        free = self.__dict__.setdefault("_free", [])
        for i, b in enumerate(free):
            if C.sizeof(b) >= size:
                return free.pop(i)
        # at least one byte: an anonymous mapping of length 0 raises ValueError before the C library
        # could report the invalid request (empty batch, trace length with no size bound)
        size = max(size, 1)
        return (C.c_char * size).from_buffer(_anon_map(size))

    def prepare(self, count, trace_length=64, buffers=0):
        """allocate workspaces for batches of `count` proofs of this shape (setup, untimed), and
        `buffers` host output buffers for submit_batch, their pages touched now -- as many as the
        caller keeps batches in flight, so steady-state submissions allocate nothing"""
        o = self._options._c()
        st = _lib.xfg_prepare(self._ctx, count, trace_length, C.byref(o))
        if st:
            raise self._err(st)
        if buffers:
            size = _lib.xfg_proof_size_bound(trace_length, C.byref(o)) * count
            free = self.__dict__.setdefault("_free", [])
            have = sum(1 for b in free if C.sizeof(b) >= size)
            for _ in range(max(0, buffers - have)):
                b = (C.c_char * size).from_buffer(_anon_map(size))
                C.memset(b, 0, size)  # fault the pages in at setup
                free.append(b)

    # ---- instrumentation
    def set_timing(self, on=True):
        _lib.xfg_set_timing(self._ctx, 1 if on else 0)

    def stage_times(self):
        ms = (C.c_double * 16)()
        names = (C.c_char_p * 16)()
        k = _lib.xfg_stage_times(self._ctx, ms, names, 16)
        return {names[i].decode(): ms[i] for i in range(k)}

    def bench_lde(self, count, n, blowup, iters):
        avg = C.c_double()
        st = _lib.xfg_bench_lde(self._ctx, count, n, blowup, iters, C.byref(avg))
        if st:
            raise self._err(st)
        return avg.value

    def lde_probe(self, enabled):
        """(total ms, launch sets, polynomials) of the trace-LDE launch sets timed in the proving
        pipeline since the last lde_probe(True) (HIP events on the launching lane's stream)"""
        ms, sets, polys = C.c_double(), C.c_uint64(), C.c_uint64()
        st = _lib.xfg_lde_probe(self._ctx, 1 if enabled else 0, C.byref(ms), C.byref(sets), C.byref(polys))
        if st:
            raise self._err(st)
        return ms.value, sets.value, polys.value

    def debug_lde(self, coef, n, blowup):
        import numpy as np
        c = np.ascontiguousarray(np.asarray(coef, dtype=np.uint64)).reshape(-1, n)
        out = np.zeros((c.shape[0], n * blowup), dtype=np.uint64)
        st = _lib.xfg_debug_lde(self._ctx, c.ctypes.data_as(_u64p), c.shape[0], n, blowup, out.ctypes.data_as(_u64p))
        if st:
            raise self._err(st)
        return out

    def debug_ood_deep(self, coef, hcoef, zpts, coeffs):
        """OOD + DEEP kernels: coef [B,7,n], hcoef [B,n], zpts [B,2], coeffs [B,8] -> (ood [B,15], deep [B,n])"""
        import numpy as np
        c = np.ascontiguousarray(coef, dtype=np.uint64)
        B, _, n = c.shape
        hc = np.ascontiguousarray(hcoef, dtype=np.uint64)
        zp = np.ascontiguousarray(zpts, dtype=np.uint64)
        co = np.ascontiguousarray(coeffs, dtype=np.uint64)
        ood = np.zeros((B, 15), dtype=np.uint64)
        deep = np.zeros((B, n), dtype=np.uint64)
        p = lambda a: a.ctypes.data_as(_u64p)
        st = _lib.xfg_debug_ood_deep(self._ctx, B, n, p(c), p(hc), p(zp), p(co), p(ood), p(deep))
        if st:
            raise self._err(st)
        return ood, deep

    FIELD_OPS = {"mul": 0, "add": 1, "sub": 2, "canon": 3, "pow2": 4, "fold": 5, "sub_weak": 6, "add_w": 7, "mul2": 8}

    def debug_field(self, op, a, b):
        """device Goldilocks primitive `op` (FIELD_OPS) applied elementwise to u64 arrays a, b"""
        import numpy as np
        x = np.ascontiguousarray(a, dtype=np.uint64)
        y = np.ascontiguousarray(b, dtype=np.uint64)
        out = np.zeros_like(x)
        st = _lib.xfg_debug_field(self._ctx, self.FIELD_OPS[op], x.size, x.ctypes.data_as(_u64p),
                                  y.ctypes.data_as(_u64p), out.ctypes.data_as(_u64p))
        if st:
            raise self._err(st)
        return out

    def debug_coin_draws(self, seed, counter, k, ext=1, reject=(0, 0, 0, 0)):
        """device transcript draws (xfg_debug_coin_draws): seed = 32 bytes, k <= 64 draws of E by one
        wave and one at a time, with counters 1..256 force-rejected where `reject` (4 x u64 bits) is
        set. Returns (wave [k][2], sequential [k][2], counters (wave, seq), ok (wave, seq))"""
        import numpy as np
        w = (C.c_uint32 * 8)(*np.frombuffer(bytes(seed), dtype="<u4").tolist())
        rej = np.array(reject, dtype=np.uint64)
        ow = np.zeros((k, 2), dtype=np.uint64)
        osq = np.zeros((k, 2), dtype=np.uint64)
        ctr = np.zeros(2, dtype=np.uint64)
        ok = (C.c_int * 2)()
        st = _lib.xfg_debug_coin_draws(self._ctx, w, counter, k, ext, rej.ctypes.data_as(_u64p),
                                       ow.ctypes.data_as(_u64p), osq.ctypes.data_as(_u64p),
                                       ctr.ctypes.data_as(_u64p), ok)
        if st:
            raise self._err(st)
        return ow, osq, (int(ctr[0]), int(ctr[1])), (ok[0], ok[1])

    def debug_interpolate(self, evals, n, offset7=False):
        import numpy as np
        e = np.ascontiguousarray(np.asarray(evals, dtype=np.uint64)).reshape(-1, n)
        out = np.zeros_like(e)
        st = _lib.xfg_debug_interpolate(self._ctx, e.ctypes.data_as(_u64p), e.shape[0], n, 1 if offset7 else 0,
                                        out.ctypes.data_as(_u64p))
        if st:
            raise self._err(st)
        return out
