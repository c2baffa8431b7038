"""ctypes binding of libkmeranno.so (include/kmeranno.h) for tests and bench.py.

The library is the product; this module only marshals numpy buffers (host entry points) or
raw device pointers (the ``*_device`` entry points, e.g. torch tensors' ``data_ptr()``).
There is no CPU fallback: if the shared library is missing or no HIP device is usable,
calls raise ``KmerAnnoError``.
"""

from __future__ import annotations

import contextlib
import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_PATH = os.environ.get("KMERANNO_LIB") or os.path.join(PKG_ROOT, "build", "libkmeranno.so")

OK = 0
E_INVALID, E_DEVICE, E_NOMEM, E_CAPACITY, E_ALPHABET, E_TABLE_FULL = -1, -2, -3, -4, -5, -6
E_IO = -7
STATUS_NONE, STATUS_CALLED, STATUS_AMBIGUOUS, STATUS_BELOW_MIN = 0, 1, 2, 3
F_END_EXCLUSIVE, F_MULTISET = 0x1, 0x2
MAX_K = 12  # K <= 8: narrow tables (8-byte slots); 9..12: wide tables (16-byte slots)

# Every symbol include/kmeranno.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "kma_abi_version", "kma_last_error", "kma_device_count", "kma_pack_kmers",
    "kma_table_create", "kma_table_create_packed", "kma_table_info_get", "kma_table_destroy",
    "kma_table_buckets_for", "kma_table_build_device", "kma_table_wrap_device",
    "kma_table_device_ptr", "kma_workspace_create", "kma_workspace_reserve",
    "kma_workspace_destroy", "kma_workspace_timing", "kma_workspace_timing_read",
    "kma_annotate_proteins", "kma_annotate_proteins_device", "kma_annotate_contigs",
    "kma_workspace_reserve_contigs", "kma_annotate_contigs_device", "kma_contig_window_count",
    "kma_peg_table_create", "kma_connect_pegs", "kma_build_signatures", "kma_table_layout_for",
    "kma_table_create_replicated", "kma_table_replicate", "kma_table_replicas",
    "kma_bucket_slots", "kma_protein_distances", "kma_protein_best_match",
    "kma_workspace_reserve_batch", "kma_workspace_phases_read", "kma_propose_pegs",
    "kma_hash_annotate", "kma_bucket_slots_for", "kma_table_buckets_for_k",
    "kma_option_set", "kma_option_get", "kma_workspace_option_set",
    "kma_packed_bytes", "kma_pack_residues", "kma_annotate_packed_device",
    "kma_table_create_from_tsv", "kma_free",
)

# Tuning options (include/kmeranno.h "options"): library-wide defaults read per call.
OPT_LAYOUT, OPT_BLOCK_PROTEINS, OPT_DEFER, OPT_HOST_PIECES, OPT_HASH_SLICE = 1, 2, 3, 4, 5
OPT_PACKED_INPUT, OPT_HOST_THREADS, OPT_HOST_SLICE, OPT_PLACEMENT = 6, 7, 8, 9
OPT_HOST_PIECE_MIN = 10
OPT_DEFAULTS = {OPT_LAYOUT: -1, OPT_BLOCK_PROTEINS: 0, OPT_DEFER: -1, OPT_HOST_PIECES: 0,
                OPT_HASH_SLICE: 0, OPT_PACKED_INPUT: 1, OPT_HOST_THREADS: 0, OPT_HOST_SLICE: 0,
                OPT_PLACEMENT: -1, OPT_HOST_PIECE_MIN: 0}
LAYOUT_TWO_CHOICE = 0x100  # layout code flag: two-choice placement (include/kmeranno.h)
LAYOUT_MOD_SAMPLING = 0x40  # layout code flag: the mod-sampling minimizer order (K = 8, m = 6)
OPT_DEFAULT = -(1 << 63)  # kma_workspace_option_set: follow the library default
_OPT_NAMES = {"layout": OPT_LAYOUT, "block_proteins": OPT_BLOCK_PROTEINS, "defer": OPT_DEFER,
              "host_pieces": OPT_HOST_PIECES, "hash_slice": OPT_HASH_SLICE,
              "packed_input": OPT_PACKED_INPUT, "host_threads": OPT_HOST_THREADS,
              "host_slice": OPT_HOST_SLICE, "placement": OPT_PLACEMENT,
              "host_piece_min": OPT_HOST_PIECE_MIN}


class KmerAnnoError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"kmeranno error {code}: {msg}")
        self.code = code


class TableInfo(C.Structure):
    _fields_ = [("n_rows", C.c_uint64), ("n_skipped", C.c_uint64), ("n_entries", C.c_uint64),
                ("n_buckets", C.c_uint64), ("bytes", C.c_uint64), ("k", C.c_int32),
                ("device", C.c_int32), ("max_probe", C.c_uint32), ("n_extra_syms", C.c_uint32),
                ("extra_syms", C.c_uint8 * 4), ("minimizer_len", C.c_int32),
                ("n_displaced", C.c_uint64), ("n_replicas", C.c_int32),
                ("slots_per_bucket", C.c_int32), ("replicate_ms", C.c_double),
                ("replicate_bytes", C.c_uint64), ("two_choice", C.c_int32),
                ("minimizer_order", C.c_int32), ("replicate_peer", C.c_int32),
                ("replicate_local", C.c_int32)]


HIT_DTYPE = np.dtype([("contig", "<u4"), ("left", "<i4"), ("fid", "<u4"), ("strand", "u1"),
                      ("frame", "u1"), ("pad", "<u2")])
PROPOSAL_DTYPE = np.dtype([("peg", "<u4"), ("contig", "<u4"), ("left", "<i4"), ("right", "<i4"),
                           ("evidence", "<u4"), ("strand", "u1"), ("frame", "u1"),
                           ("pad", "<u2")])

_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C")
_vp, _u64, _u32, _int = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
_lib = None


def load(path: str | None = None):
    """Load libkmeranno.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is None:
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise KmerAnnoError(E_DEVICE, f"{p} not built (run `make -C kmers.anno_amd`)")
        L = C.CDLL(p)
        L.kma_last_error.restype = C.c_char_p
        L.kma_device_count.argtypes = [C.POINTER(C.c_int)]
        L.kma_pack_kmers.argtypes = [_vp, C.c_char_p, _u64p, _u64, _u64p]
        L.kma_table_create.argtypes = [C.c_char_p, _u64p, _u32p, _u64, _int, _int, C.c_double,
                                       C.POINTER(_vp)]
        L.kma_table_create_packed.argtypes = [_u64p, _u32p, _u64, _int, _int, C.c_double,
                                              C.POINTER(_vp)]
        L.kma_table_info_get.argtypes = [_vp, C.POINTER(TableInfo)]
        L.kma_table_destroy.argtypes = [_vp]
        L.kma_table_buckets_for.restype = _u64
        L.kma_table_buckets_for.argtypes = [_u64, C.c_double]
        L.kma_table_buckets_for_k.restype = _u64
        L.kma_table_buckets_for_k.argtypes = [_u64, C.c_double, _int]
        L.kma_bucket_slots_for.argtypes = [_int]
        L.kma_table_build_device.argtypes = [_vp, _u64, _int, _int, _vp, _vp, _vp, _u64, _vp,
                                             _vp]
        L.kma_table_wrap_device.argtypes = [_vp, _u64, _int, _int, _int, C.POINTER(_vp)]
        L.kma_table_layout_for.argtypes = [_int, _u64]
        L.kma_protein_distances.argtypes = [_u8p, _u64p, _u32, _int, _u32, _u32p, _u32p, _u64,
                                            _int, _u32p, _vp, _vp]
        L.kma_protein_best_match.argtypes = [_u8p, _u64p, _u32, _int, _u32, _u32p, _u64p, _u32p,
                                             _u32, C.c_double, _int, _i32p, _vp]
        L.kma_table_create_replicated.argtypes = [C.c_char_p, _u64p, _u32p, _u64, _int, _int,
                                                  _i32p, C.c_double, C.POINTER(_vp)]
        L.kma_table_replicate.argtypes = [_vp, _int, _i32p]
        L.kma_table_create_from_tsv.argtypes = [C.c_char_p, _int, _int, _i32p, C.c_double,
                                                C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_u64),
                                                C.POINTER(_u32), C.POINTER(_int)]
        L.kma_free.argtypes = [_vp]
        L.kma_free.restype = None
        L.kma_table_replicas.argtypes = [_vp, C.POINTER(_int), _vp, _int]
        L.kma_table_device_ptr.argtypes = [_vp, C.POINTER(_vp), C.POINTER(_u64)]
        L.kma_workspace_create.argtypes = [_int, C.POINTER(_vp)]
        L.kma_workspace_destroy.argtypes = [_vp]
        L.kma_workspace_reserve.argtypes = [_vp, _u64]
        L.kma_workspace_timing.argtypes = [_vp, _int]
        L.kma_workspace_timing_read.argtypes = [_vp, C.POINTER(_u32), C.POINTER(C.c_double),
                                                C.POINTER(C.c_double)]
        L.kma_workspace_reserve_batch.argtypes = [_vp, _u64, _u64]
        L.kma_workspace_phases_read.argtypes = [_vp, C.POINTER(_u32), C.POINTER(_int),
                                                C.POINTER(C.c_double), C.POINTER(C.c_char_p)]
        L.kma_annotate_proteins.argtypes = [_vp, _u8p, _u64p, _u32, _int, _u32, _i32p, _i32p,
                                            _u8p, _vp, _u32]
        L.kma_annotate_proteins_device.argtypes = [_vp, _vp, _vp, _vp, _u32, _u64, _int, _u32,
                                                   _vp, _vp, _vp, _vp, _u32, _vp]
        L.kma_annotate_contigs.argtypes = [_vp, _u8p, _u64p, _u32, _int, _vp, _u64,
                                           C.POINTER(_u64), _vp, _u32]
        L.kma_workspace_reserve_contigs.argtypes = [_vp, _u64]
        L.kma_annotate_contigs_device.argtypes = [_vp, _vp, _vp, _vp, _u32, _u64, _int, _vp,
                                                  _u64, _vp, _vp, _u32, _vp]
        L.kma_build_signatures.argtypes = [_u8p, _u64p, _i32p, _u32, _int, _u32, _int, _vp, _vp,
                                           _u64, C.POINTER(_u64)]
        L.kma_peg_table_create.argtypes = [_u8p, _u64p, _u32, _int, _int, C.c_double,
                                           C.POINTER(_vp), C.POINTER(_u64)]
        L.kma_connect_pegs.argtypes = [_vp, _u8p, _u64p, _u32, _int, _int, _vp, _u64,
                                       C.POINTER(_u64)]
        L.kma_hash_annotate.argtypes = [_u8p, _u64p, _u32, _u8p, _u64p, _u32, _int, C.c_double,
                                        _int, _vp, _vp, _vp]
        L.kma_propose_pegs.argtypes = [_vp, _u64, _u32p, _u32, _int, C.c_double, C.c_double,
                                       C.c_double, _int, _vp, _u64, C.POINTER(_u64), _u64p]
        L.kma_contig_window_count.restype = _u64
        L.kma_contig_window_count.argtypes = [_u64p, _u32, _int]
        L.kma_option_set.argtypes = [_int, C.c_int64]
        L.kma_option_get.argtypes = [_int, C.POINTER(C.c_int64)]
        L.kma_workspace_option_set.argtypes = [_vp, _int, C.c_int64]
        L.kma_packed_bytes.restype = _u64
        L.kma_packed_bytes.argtypes = [_u64]
        L.kma_pack_residues.argtypes = [_vp, _u8p, _u64, _u8p, _u64]
        L.kma_annotate_packed_device.argtypes = [_vp, _vp, _vp, _vp, _u32, _u64, _int, _u32,
                                                 _vp, _vp, _vp, _vp, _u32, _vp]
        _lib = L
    return _lib


def _check(rc: int):
    if rc != OK:
        raise KmerAnnoError(rc, load().kma_last_error().decode(errors="replace"))


def set_option(option: int, value: int):
    """Library-wide tuning default (OPT_* ; see include/kmeranno.h)."""
    _check(load().kma_option_set(option, int(value)))


def get_option(option: int) -> int:
    v = C.c_int64()
    _check(load().kma_option_get(option, C.byref(v)))
    return v.value


def reset_options():
    for o, v in OPT_DEFAULTS.items():
        set_option(o, v)


@contextlib.contextmanager
def options(**kw):
    """Set options by name (layout=, block_proteins=, defer=, host_pieces=, hash_slice=) for
    the body, then restore the previous values."""
    old = {_OPT_NAMES[k]: get_option(_OPT_NAMES[k]) for k in kw}
    try:
        for k, v in kw.items():
            set_option(_OPT_NAMES[k], v)
        yield
    finally:
        for o, v in old.items():
            set_option(o, v)


def source_digest() -> str:
    """sha256[:16] of the native sources (csrc/ and the ABI header): stamps counter summaries
    under profiles/ so that a bench run can tell whether they describe the kernels it runs."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(PKG_ROOT, "csrc")
    hdr = os.path.join(os.path.dirname(PKG_ROOT), "include", "kmeranno.h")
    for f in sorted(os.listdir(csrc)) + [hdr]:
        path = f if os.path.isabs(f) else os.path.join(csrc, f)
        if os.path.isfile(path):
            h.update(os.path.basename(path).encode())
            h.update(open(path, "rb").read())
    return h.hexdigest()[:16]


def device_count() -> int:
    n = C.c_int(0)
    _check(load().kma_device_count(C.byref(n)))
    return n.value


def pack_strings(strs):
    """Concatenate strings -> (uint8 buffer padded by 32 bytes, uint64 offsets)."""
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strs]
    offsets = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        offsets[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bs) + b"\0" * 32, dtype=np.uint8).copy()
    return buf, offsets


def std_codes(ascii_bytes: np.ndarray) -> np.ndarray:
    """Standard 5-bit residue codes ('A'..'Z' -> 1..26, '*' -> 27, other -> 0)."""
    b = ascii_bytes.astype(np.int64)
    c = np.where((b >= 65) & (b <= 90), b - 64, 0)
    return np.where(b == 42, 27, c).astype(np.uint64)


def pack_std(kmers_u8: np.ndarray) -> np.ndarray:
    """Pack an (n, k) uint8 array of ASCII kmers into keys (standard alphabet, 0 if invalid)."""
    codes = std_codes(kmers_u8)
    k = kmers_u8.shape[1]
    keys = np.zeros(len(kmers_u8), np.uint64)
    for j in range(k):
        keys = (keys << np.uint64(5)) | codes[:, j]
    keys[(codes == 0).any(axis=1)] = 0
    return keys


class SignatureTable:
    """A signature table resident on one GPU (ApplyKmerProcessor.java:100-110)."""

    def __init__(self, handle, owner=True):
        self._h = handle
        self._owner = owner

    @classmethod
    def from_rows(cls, kmers, fids, k: int = 8, device: int = 0, load_factor: float = 0.5):
        buf, off = pack_strings(kmers)
        h = _vp()
        _check(load().kma_table_create(buf.tobytes(), off, np.ascontiguousarray(fids, np.uint32),
                                       len(off) - 1, k, device, load_factor, C.byref(h)))
        return cls(h)

    @classmethod
    def from_packed(cls, keys, fids, k: int = 8, device: int = 0, load_factor: float = 0.5):
        keys = np.ascontiguousarray(keys, np.uint64)
        h = _vp()
        _check(load().kma_table_create_packed(keys, np.ascontiguousarray(fids, np.uint32),
                                              len(keys), k, device, load_factor, C.byref(h)))
        return cls(h)

    @classmethod
    def from_pegs(cls, residues, offsets, k: int = 8, device: int = 0, load_factor: float = 0.5):
        """Singleton peg-kmer table of a close genome (fid = peg index); see kma_peg_table_create.
        Returns (table, counted windows)."""
        residues = np.ascontiguousarray(residues, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        h, nw = _vp(), _u64()
        _check(load().kma_peg_table_create(residues, offsets, len(offsets) - 1, k, device,
                                           load_factor, C.byref(h), C.byref(nw)))
        return cls(h), nw.value

    @classmethod
    def from_rows_replicated(cls, kmers, fids, devices, k: int = 8, load_factor: float = 0.5):
        """One table with a replica on each listed device (a device may repeat); host calls
        shard their batch over the replicas."""
        buf, off = pack_strings(kmers)
        dv = np.ascontiguousarray(devices, np.int32)
        h = _vp()
        _check(load().kma_table_create_replicated(buf.tobytes(), off,
                                                  np.ascontiguousarray(fids, np.uint32),
                                                  len(off) - 1, k, len(dv), dv, load_factor,
                                                  C.byref(h)))
        return cls(h)

    @classmethod
    def from_tsv(cls, path: str, k: int = 8, devices=(0,), load_factor: float = 0.5):
        """The table of apply's kmerdb.tbl read by the library (kma_table_create_from_tsv):
        returns (table, role ids in fid order, the last row's kmer length)."""
        dv = np.ascontiguousarray(devices, np.int32)
        h, names, nb, nr, last = _vp(), _vp(), _u64(), _u32(), _int()
        _check(load().kma_table_create_from_tsv(os.fsencode(path), k, len(dv), dv, load_factor,
                                                C.byref(h), C.byref(names), C.byref(nb),
                                                C.byref(nr), C.byref(last)))
        try:
            blob = C.string_at(names.value, nb.value) if nb.value else b""
        finally:
            load().kma_free(names)
        roles = [r.decode() for r in blob.split(b"\0")[:-1]] if blob else []
        assert len(roles) == nr.value
        return cls(h), roles, last.value

    @classmethod
    def wrap_device(cls, d_slots: int, n_buckets: int, k: int = 8, device: int = 0,
                    layout: int = -1):
        h = _vp()
        _check(load().kma_table_wrap_device(d_slots, n_buckets, k, layout, device, C.byref(h)))
        return cls(h)

    def replicate(self, devices):
        dv = np.ascontiguousarray(devices, np.int32)
        _check(load().kma_table_replicate(self._h, len(dv), dv))

    @property
    def replicas(self):
        n = _int(0)
        _check(load().kma_table_replicas(self._h, C.byref(n), None, 0))
        out = (C.c_int * max(n.value, 1))()
        _check(load().kma_table_replicas(self._h, C.byref(n), out, n.value))
        return list(out)[:n.value]

    @property
    def info(self) -> TableInfo:
        i = TableInfo()
        _check(load().kma_table_info_get(self._h, C.byref(i)))
        return i

    def device_ptr(self):
        p, n = _vp(), _u64()
        _check(load().kma_table_device_ptr(self._h, C.byref(p), C.byref(n)))
        return p.value, n.value

    def pack(self, kmers) -> np.ndarray:
        buf, off = pack_strings(kmers)
        out = np.zeros(len(off) - 1, np.uint64)
        _check(load().kma_pack_kmers(self._h, buf.tobytes(), off, len(off) - 1, out))
        return out

    def close(self):
        if self._h:
            load().kma_table_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Workspace:
    def __init__(self, device: int = 0, n_residues: int = 0, n_seq: int = 0):
        self._h = _vp()
        _check(load().kma_workspace_create(device, C.byref(self._h)))
        if n_residues:
            self.reserve(n_residues, n_seq)

    def reserve(self, n_residues: int, n_seq: int = 0):
        """Scratch for device calls of up to n_residues residues and n_seq proteins (0: the
        library's default of n_residues / 16 + 256)."""
        if n_seq:
            _check(load().kma_workspace_reserve_batch(self._h, n_residues, n_seq))
        else:
            _check(load().kma_workspace_reserve(self._h, n_residues))

    def reserve_contigs(self, n_bases: int):
        _check(load().kma_workspace_reserve_contigs(self._h, n_bases))

    def set_option(self, option: int, value: int = OPT_DEFAULT):
        """Per-workspace override of OPT_BLOCK_PROTEINS / OPT_DEFER (OPT_DEFAULT: none)."""
        _check(load().kma_workspace_option_set(self._h, option, int(value)))

    def timing(self, enable: bool = True):
        """Per-phase hipEvent timing of the device calls made with this workspace."""
        _check(load().kma_workspace_timing(self._h, int(enable)))

    def timing_read(self):
        """(n_calls, kernel_ms_total, rest_ms_total) since the last read; clears them."""
        n, p, v = _u32(), C.c_double(), C.c_double()
        _check(load().kma_workspace_timing_read(self._h, C.byref(n), C.byref(p), C.byref(v)))
        return n.value, p.value, v.value

    def phases_read(self):
        """(n_calls, {phase name: summed ms}) of the calls laid out like the last one (same
        path) since the last read; clears them."""
        n, k = _u32(), _int()
        ms = (C.c_double * 8)()
        names = (C.c_char_p * 8)()
        _check(load().kma_workspace_phases_read(self._h, C.byref(n), C.byref(k), ms, names))
        return n.value, {names[i].decode(): ms[i] for i in range(k.value)}

    def close(self):
        if self._h:
            load().kma_workspace_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def buckets_for(n_keys: int, load_factor: float = 0.5, k: int = 8) -> int:
    return int(load().kma_table_buckets_for_k(n_keys, load_factor, k))


def bucket_slots(k: int = 8) -> int:
    """Slots per bucket of a table of k-mers: narrow (k <= 8) u64 slots of this build (8: 64-byte
    buckets; 16: the 128-byte variant), wide (k 9..12) 4 slots of 16 bytes."""
    return int(load().kma_bucket_slots_for(k))


def layout_for(k: int, n_buckets: int) -> int:
    """The size-derived table layout code (minimizer length, 0 = flat; | LAYOUT_TWO_CHOICE when
    the creators try two-choice placement first)."""
    return int(load().kma_table_layout_for(k, n_buckets))


# The creators' layout rule by measurement (kma_internal.h kRetryDisplaced / kMaxDisplaced /
# kMaxChain / kMaxDisplacedTwoChoice; kma_abi.cpp create_from_device_keys).
RETRY_DISPLACED, MAX_DISPLACED, MAX_CHAIN = 0.10, 0.15, 32
MAX_DISPLACED_TWO_CHOICE = 0.40


def choose_layout(k: int, n_buckets: int, build):
    """The library creators' layout choice for hosts that build tables on the device
    themselves (kma_table_build_device into their own buffer, e.g. one RCCL broadcasts):
    build(code) builds the table with that layout code (minimizer length | LAYOUT_TWO_CHOICE)
    into the caller's buffer and returns its status {failed, entries, longest chain,
    displaced}. Returns (code, status); the kept layout is the one built last. Two-choice
    placement first (narrow tables; a failed minimizer build is retried flat); a failed
    two-choice build falls back to the chained rule.
    A forced layout (OPT_LAYOUT) is the size rule's answer."""
    def disp(s):
        return s[3] / max(s[1], 1)
    forced = get_option(OPT_LAYOUT) != -1
    code = layout_for(k, n_buckets)
    m = code & 0xFF
    if code & LAYOUT_TWO_CHOICE:
        st = build(code)
        if st[0] != 0 and m != 0 and not forced:  # out of evictions: retried flat
            s2 = build(LAYOUT_TWO_CHOICE)
            if s2[0] == 0:
                return LAYOUT_TWO_CHOICE, s2
        if st[0] == 0:
            if not forced and m != 0 and disp(st) > MAX_DISPLACED_TWO_CHOICE:
                s2 = build(LAYOUT_TWO_CHOICE)
                if s2[0] == 0 and 2 * s2[3] < st[3]:
                    return LAYOUT_TWO_CHOICE, s2
                st = build(code)
            return code, st
    st = build(m)
    if forced:
        return m, st
    m6, m7 = min(k, 6), min(k, 7)
    if m & 0x3F == m6 and m6 != m7 and disp(st) > RETRY_DISPLACED:
        s2 = build(m7)
        if s2[3] < st[3]:
            m, st = m7, s2
        else:
            st = build(m)
    if m != 0 and (disp(st) > MAX_DISPLACED or st[2] > MAX_CHAIN):
        s2 = build(0)
        if 2 * s2[3] < st[3] or (st[2] > MAX_CHAIN and 2 * s2[2] < st[2]):
            m, st = 0, s2
        else:
            st = build(m)
    return m, st


def build_device(d_slots: int, n_buckets: int, d_winner: int, d_keys: int, d_fids: int, n: int,
                 d_status: int, stream: int = 0, k: int = 8, layout: int = -1):
    """Device-resident table build; d_status (4 x u32) <- {full, entries, longest chain,
    displaced keys}."""
    _check(load().kma_table_build_device(d_slots, n_buckets, k, layout, d_winner, d_keys, d_fids,
                                         n, d_status, stream or None))


def annotate_proteins(table: SignatureTable, residues: np.ndarray, offsets: np.ndarray,
                      min_hits: int = 5, flags: int = 0, n_fid: int = 0, out=None):
    """Host form of the apply loop: returns (fid, count, status, tally-or-None). out: the
    caller's (fid, count, status[, tally]) arrays to fill (reused buffers, as a JNI caller
    passes its direct buffers: fresh arrays cost their first-touch page faults)."""
    residues = np.ascontiguousarray(residues, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets) - 1
    if out is not None:
        fid, cnt, st = out[:3]
        assert fid.dtype == np.int32 and cnt.dtype == np.int32 and st.dtype == np.uint8
        assert len(fid) == len(cnt) == len(st) == n and fid.flags.c_contiguous
        tally = (out[3] if len(out) > 3 else np.zeros(n_fid, np.uint32)) if n_fid else None
        if tally is not None:
            tally[:] = 0
    else:
        fid, cnt, st = np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.uint8)
        tally = np.zeros(n_fid, np.uint32) if n_fid else None
    _check(load().kma_annotate_proteins(table._h, residues, offsets, n, min_hits, flags, fid, cnt,
                                        st, tally.ctypes.data if n_fid else None, n_fid))
    return fid, cnt, st, tally


def annotate_proteins_device(table: SignatureTable, ws: Workspace, d_residues: int,
                             d_offsets: int, n_seq: int, n_residues: int, min_hits: int,
                             flags: int, d_fid: int, d_count: int, d_status: int, d_tally: int = 0,
                             n_fid: int = 0, stream: int = 0):
    _check(load().kma_annotate_proteins_device(table._h, ws._h, d_residues, d_offsets, n_seq,
                                               n_residues, min_hits, flags, d_fid, d_count,
                                               d_status, d_tally or None, n_fid, stream or None))


HOST_PROFILE_FIELDS = ("setup_ms", "stage_ms", "launch_ms", "wait_ms", "outputs_ms", "call_ms",
                       "staging_threads", "pieces")


def host_profile(replica: int | None = None) -> dict:
    """The library's host-side phase profile (measurement hook, not in kmeranno.h) of the last
    host protein shard call, or of replica `replica`'s last shard of a fanned-out call."""
    L = load()
    p = (C.c_double * len(HOST_PROFILE_FIELDS))()
    if replica is None:
        _check(L.kma_debug_host_profile(p, len(p)))
    else:
        _check(L.kma_debug_host_profile_replica(replica, p, len(p)))
    return dict(zip(HOST_PROFILE_FIELDS, list(p)))


def host_cores() -> int:
    """CPUs the library sizes its staging jobs by (affinity mask bounded by the cgroup quota)."""
    return int(load().kma_debug_host_cores())


def packed_bytes(n_residues: int) -> int:
    return int(load().kma_packed_bytes(n_residues))


def pack_residues(table, residues: np.ndarray, n: int | None = None) -> np.ndarray:
    """The packed residue stream (5 bits per residue, the table's codes; table None: the
    standard alphabet) of residues[0, n)."""
    residues = np.ascontiguousarray(residues, np.uint8)
    n = len(residues) if n is None else n
    out = np.empty(packed_bytes(n), np.uint8)
    _check(load().kma_pack_residues(table._h if table is not None else None, residues, n, out,
                                    len(out)))
    return out


def annotate_packed_device(table: SignatureTable, ws: Workspace, d_stream: int, d_offsets: int,
                           n_seq: int, n_residues: int, min_hits: int, flags: int, d_fid: int,
                           d_count: int, d_status: int, d_tally: int = 0, n_fid: int = 0,
                           stream: int = 0):
    _check(load().kma_annotate_packed_device(table._h, ws._h, d_stream, d_offsets, n_seq,
                                             n_residues, min_hits, flags, d_fid, d_count,
                                             d_status, d_tally or None, n_fid, stream or None))


def annotate_contigs(table: SignatureTable, dna: np.ndarray, offsets: np.ndarray,
                     genetic_code: int = 11, n_fid: int = 0):
    """6-frame annotation: returns (hits structured array, tally[n_contig, n_fid] or None)."""
    dna = np.ascontiguousarray(dna, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n_contig = len(offsets) - 1
    cap = max(1024, int(load().kma_contig_window_count(offsets, n_contig, table.info.k)) // 8)
    while True:
        hits = np.empty(cap, HIT_DTYPE)
        tally = np.zeros((n_contig, n_fid), np.uint32) if n_fid else None
        nh = _u64()
        rc = load().kma_annotate_contigs(table._h, dna, offsets, n_contig, genetic_code,
                                         hits.ctypes.data, cap, C.byref(nh),
                                         tally.ctypes.data if n_fid else None, n_fid)
        if rc == E_CAPACITY:
            cap = nh.value
            continue
        _check(rc)
        return hits[:nh.value], tally


def annotate_contigs_device(table: SignatureTable, ws: Workspace, d_dna: int, d_offsets: int,
                            n_contig: int, n_bases: int, genetic_code: int, d_hits: int, cap: int,
                            d_n_hits: int, d_tally: int = 0, n_fid: int = 0, stream: int = 0):
    """Device form of the 6-frame pass (asynchronous on `stream`; *d_n_hits gets the total)."""
    _check(load().kma_annotate_contigs_device(table._h, ws._h, d_dna, d_offsets, n_contig,
                                              n_bases, genetic_code, d_hits or None, cap,
                                              d_n_hits, d_tally or None, n_fid, stream or None))


def connect_pegs(peg_table: SignatureTable, dna: np.ndarray, offsets: np.ndarray,
                 genetic_code: int = 11, strict: bool = False):
    """KmerProcessor.java:195-207: (hits with fid = peg index) in canonical order."""
    dna = np.ascontiguousarray(dna, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n_contig = len(offsets) - 1
    cap = 1024
    while True:
        hits = np.empty(cap, HIT_DTYPE)
        nh = _u64()
        rc = load().kma_connect_pegs(peg_table._h, dna, offsets, n_contig, genetic_code,
                                     int(strict), hits.ctypes.data, cap, C.byref(nh))
        if rc == E_CAPACITY:
            cap = nh.value
            continue
        _check(rc)
        return hits[:nh.value]


def propose_pegs(hits: np.ndarray, peg_len, k: int = 8, min_strength: float = 0.5,
                 max_fuzz: float = 1.5, min_fuzz: float = 0.8, device: int = 0):
    """KmerProcessor.java:209-264 on the GPU: the proposal sweep over the framed location lists
    of connect_pegs' hits (fid = peg index). Returns (PROPOSAL_DTYPE array, stats[4] =
    lists, too few kmers, too short, proposals)."""
    hits = np.ascontiguousarray(hits, HIT_DTYPE)
    peg_len = np.ascontiguousarray(peg_len, np.uint32)
    stats = np.zeros(4, np.uint64)
    cap = max(16, len(hits) // 4)
    while True:
        out = np.empty(cap, PROPOSAL_DTYPE)
        n = _u64()
        rc = load().kma_propose_pegs(hits.ctypes.data if len(hits) else None, len(hits), peg_len,
                                     len(peg_len), k, min_strength, max_fuzz, min_fuzz, device,
                                     out.ctypes.data, cap, C.byref(n), stats)
        if rc == E_CAPACITY:
            cap = n.value
            continue
        _check(rc)
        return out[:n.value], stats


def hash_annotate(genome_residues, genome_offsets, proto_residues, proto_offsets, k: int = 8,
                  min_sim: float = 0.0125, device: int = 0):
    """HashAnnotationProcessor.java:233-306 scoring on the GPU: (best prototype per genome
    protein or -1, its similarity (0.0 if none), matches per prototype)."""
    gr = np.ascontiguousarray(genome_residues, np.uint8)
    go = np.ascontiguousarray(genome_offsets, np.uint64)
    pr = np.ascontiguousarray(proto_residues, np.uint8)
    po = np.ascontiguousarray(proto_offsets, np.uint64)
    n_g, n_p = len(go) - 1, len(po) - 1
    best = np.empty(max(n_g, 1), np.int32)
    sim = np.empty(max(n_g, 1), np.float64)
    cnt = np.empty(max(n_p, 1), np.uint32)
    _check(load().kma_hash_annotate(gr if len(gr) else np.zeros(1, np.uint8), go, n_g,
                                    pr if len(pr) else np.zeros(1, np.uint8), po, n_p, k,
                                    min_sim, device, best.ctypes.data, sim.ctypes.data,
                                    cnt.ctypes.data))
    return best[:n_g], sim[:n_g], cnt[:n_p]


def build_signatures(residues: np.ndarray, offsets: np.ndarray, roles, k: int = 8,
                     flags: int = 0, device: int = 0):
    """BuildKmerProcessor's discriminating kmers on the GPU: (packed keys, roles), key order."""
    residues = np.ascontiguousarray(residues, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    roles = np.ascontiguousarray(roles, np.int32)
    n = len(offsets) - 1
    cap = 1 << 16
    while True:
        keys, rl, nout = np.empty(cap, np.uint64), np.empty(cap, np.uint32), _u64()
        rc = load().kma_build_signatures(residues, offsets, roles, n, k, flags, device,
                                         keys.ctypes.data, rl.ctypes.data, cap, C.byref(nout))
        if rc == E_CAPACITY:
            cap = nout.value
            continue
        _check(rc)
        return keys[:nout.value], rl[:nout.value]


def contig_window_count(offsets: np.ndarray, k: int = 8) -> int:
    offsets = np.ascontiguousarray(offsets, np.uint64)
    return int(load().kma_contig_window_count(offsets, len(offsets) - 1, k))


def protein_distances(residues, offsets, pair_a, pair_b, k: int = 8, flags: int = 0,
                      device: int = 0):
    """ProteinKmers.distance per pair (GeneCopyProcessor.java:137-142) on the GPU:
    (similarity, per-protein set sizes, distances)."""
    residues = np.ascontiguousarray(residues, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    pa = np.ascontiguousarray(pair_a, np.uint32)
    pb = np.ascontiguousarray(pair_b, np.uint32)
    n = len(offsets) - 1
    sim = np.empty(len(pa), np.uint32)
    size = np.empty(n, np.uint32)
    dist = np.empty(len(pa), np.float64)
    _check(load().kma_protein_distances(residues, offsets, n, k, flags, pa, pb, len(pa), device,
                                        sim, size.ctypes.data, dist.ctypes.data))
    return sim, size, dist


def protein_best_match(residues, offsets, query, cand_off, cand, max_dist: float, k: int = 8,
                       flags: int = 0, device: int = 0):
    """GeneCopyProcessor's closest-source choice (:135-146): (best index or -1, distance)."""
    residues = np.ascontiguousarray(residues, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    query = np.ascontiguousarray(query, np.uint32)
    cand_off = np.ascontiguousarray(cand_off, np.uint64)
    cand = np.ascontiguousarray(cand, np.uint32)
    best = np.empty(len(query), np.int32)
    bd = np.empty(len(query), np.float64)
    _check(load().kma_protein_best_match(residues, offsets, len(offsets) - 1, k, flags, query,
                                         cand_off, cand if len(cand) else np.zeros(1, np.uint32),
                                         len(query), max_dist, device, best, bd.ctypes.data))
    return best, bd

