"""ctypes loader for the C oracle (oracle/kma_oracle.c) — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It is the checker (and the CPU baseline), never the thing measured as the product.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")

_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.orc_table_new.restype = C.c_void_p
        L.orc_table_new.argtypes = [C.c_char_p, _u64p, _i32p, C.c_uint64]
        L.orc_table_free.argtypes = [C.c_void_p]
        L.orc_table_size.restype = C.c_uint64
        L.orc_table_size.argtypes = [C.c_void_p]
        L.orc_apply.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint32, C.c_int, C.c_int,
                                C.c_uint32, _i32p, _i32p, _u8p]
        L.orc_apply_mt.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint32, C.c_int, C.c_int,
                                   C.c_uint32, _i32p, _i32p, _u8p, C.c_int]
        L.orc_protein_distances.argtypes = [_u8p, _u64p, C.c_int, C.c_uint32, _u32p, _u32p,
                                            C.c_uint64, _u32p, _u32p, _u32p,
                                            np.ctypeslib.ndpointer(np.float64, flags="C")]
        L.orc_translate.restype = C.c_int64
        L.orc_translate.argtypes = [C.c_char_p, C.c_int64, C.c_int, C.c_int, C.c_char_p]
        L.orc_contig_kmers.restype = C.c_uint64
        L.orc_contig_kmers.argtypes = [_u8p, _u64p, C.c_uint32, C.c_int, C.c_int, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_uint64]
        L.orc_annotate_contigs.restype = C.c_uint64
        L.orc_annotate_contigs.argtypes = [C.c_void_p, _u8p, _u64p, C.c_uint32, C.c_int,
                                           C.c_int, _u32p, _i32p, _u8p, _u8p, _u32p,
                                           C.c_uint64]
        L.orc_peg_kmers.restype = C.c_uint64
        L.orc_peg_kmers.argtypes = [_u8p, _u64p, C.c_uint32, C.c_int, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_uint64]
        L.orc_peg_connect.restype = C.c_uint64
        L.orc_peg_connect.argtypes = [_u8p, _u64p, C.c_uint32, _u8p, _u64p, C.c_uint32, C.c_int,
                                      C.c_int, C.c_int, _u32p, _i32p, _u8p, _u8p, _u32p,
                                      C.c_uint64]
        L.orc_build.restype = C.c_uint64
        L.orc_build.argtypes = [_u8p, _u64p, _i32p, C.c_uint32, C.c_int, C.c_uint32, C.c_void_p,
                                C.c_void_p, C.c_uint64]
        _lib = L
    return _lib


def pack_strings(strs):
    """Concatenate byte strings -> (uint8 buffer padded by 16 bytes, uint64 offsets)."""
    bs = [s.encode() if isinstance(s, str) else bytes(s) for s in strs]
    offsets = np.zeros(len(bs) + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bs) + b"\0" * 32, dtype=np.uint8).copy()
    return buf, offsets


class Table:
    """HashMap<String,String> of ApplyKmerProcessor.java:101-107 (values are int role ids)."""

    def __init__(self, kmers=None, values=None, _raw=None):
        buf, off = _raw if _raw is not None else pack_strings(kmers)
        buf = buf if isinstance(buf, bytes) else buf.tobytes()
        self._h = lib().orc_table_new(buf, np.ascontiguousarray(off, np.uint64),
                                      np.ascontiguousarray(values, np.int32), len(off) - 1)
        self.size = lib().orc_table_size(self._h)

    @classmethod
    def from_buffer(cls, text: bytes, offsets: np.ndarray, values):
        """Rows text[offsets[r]:offsets[r+1]] (avoids building Python strings)."""
        return cls(values=values, _raw=(text, offsets))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_table_free(self._h)
            self._h = None


def apply(table: Table, residues: np.ndarray, offsets: np.ndarray, k: int = 8,
          min_hits: int = 5, flags: int = 0):
    n = len(offsets) - 1
    fid = np.empty(n, np.int32)
    cnt = np.empty(n, np.int32)
    st = np.empty(n, np.uint8)
    lib().orc_apply(table._h, residues, offsets, n, k, min_hits, flags, fid, cnt, st)
    return fid, cnt, st


def apply_mt(table: Table, residues: np.ndarray, offsets: np.ndarray, k: int = 8,
             min_hits: int = 5, flags: int = 0, threads: int = 1):
    """orc_apply over `threads` pthreads (contiguous protein ranges; same outputs)."""
    n = len(offsets) - 1
    fid = np.empty(n, np.int32)
    cnt = np.empty(n, np.int32)
    st = np.empty(n, np.uint8)
    lib().orc_apply_mt(table._h, residues, offsets, n, k, min_hits, flags, fid, cnt, st, threads)
    return fid, cnt, st


def translate(dna: str, frame: int, gcode: int = 11) -> str:
    out = C.create_string_buffer(len(dna) // 3 + 2)
    n = lib().orc_translate(dna.encode(), len(dna), frame, gcode, out)
    if n < 0:
        raise ValueError(f"unsupported genetic code {gcode}")
    return out.raw[:n].decode()


def contig_kmers(dna: np.ndarray, offsets: np.ndarray, gcode: int = 11, k: int = 8):
    """Records of KmerReference.getContigKmers: (kmers[n,k] bytes, contig, left, strand, frame)."""
    n_contig = len(offsets) - 1
    n = lib().orc_contig_kmers(dna, offsets, n_contig, gcode, k, None, None, None, None, None, 0)
    km = np.empty((n, k), np.uint8)
    ct = np.empty(n, np.uint32)
    lf = np.empty(n, np.int32)
    sd = np.empty(n, np.uint8)
    fr = np.empty(n, np.uint8)
    lib().orc_contig_kmers(dna, offsets, n_contig, gcode, k, km.ctypes.data, ct.ctypes.data,
                           lf.ctypes.data, sd.ctypes.data, fr.ctypes.data, n)
    return km, ct, lf, sd, fr


def annotate_contigs(table: Table, dna: np.ndarray, offsets: np.ndarray, gcode: int = 11,
                     k: int = 8):
    """Sorted hits (contig, left, strand, frame, fid) of every 6-frame window in the table."""
    n_contig = len(offsets) - 1
    z32, zi, z8 = np.empty(1, np.uint32), np.empty(1, np.int32), np.empty(1, np.uint8)
    n = lib().orc_annotate_contigs(table._h, dna, offsets, n_contig, gcode, k, z32, zi, z8, z8,
                                   z32, 0)
    ct, lf = np.empty(n, np.uint32), np.empty(n, np.int32)
    sd, fr, fid = np.empty(n, np.uint8), np.empty(n, np.uint8), np.empty(n, np.uint32)
    lib().orc_annotate_contigs(table._h, dna, offsets, n_contig, gcode, k, ct, lf, sd, fr, fid, n)
    return ct, lf, sd, fr, fid


def peg_kmers(residues: np.ndarray, offsets: np.ndarray, k: int = 8):
    n_seq = len(offsets) - 1
    n = lib().orc_peg_kmers(residues, offsets, n_seq, k, None, None, None, 0)
    km = np.empty((n, k), np.uint8)
    pg = np.empty(n, np.uint32)
    lf = np.empty(n, np.int32)
    lib().orc_peg_kmers(residues, offsets, n_seq, k, km.ctypes.data, pg.ctypes.data,
                        lf.ctypes.data, n)
    return km, pg, lf


def peg_connect(residues, offsets, dna, doffsets, gcode: int = 11, k: int = 8, strict=False):
    """Connections (contig, left, strand, frame, peg) of KmerProcessor.java:195-207, sorted."""
    args = (residues, offsets, len(offsets) - 1, dna, doffsets, len(doffsets) - 1, gcode, k,
            int(strict))
    z32, zi, z8 = np.empty(1, np.uint32), np.empty(1, np.int32), np.empty(1, np.uint8)
    n = lib().orc_peg_connect(*args, z32, zi, z8, z8, z32, 0)
    ct, lf = np.empty(n, np.uint32), np.empty(n, np.int32)
    sd, fr, pg = np.empty(n, np.uint8), np.empty(n, np.uint8), np.empty(n, np.uint32)
    lib().orc_peg_connect(*args, ct, lf, sd, fr, pg, n)
    return ct, lf, sd, fr, pg


def build_signatures(residues, offsets, roles, k: int = 8, flags: int = 0):
    """BuildKmerProcessor's discriminating kmers: (kmers[n, k] bytes, roles[n]) in table order."""
    roles = np.ascontiguousarray(roles, np.int32)
    n_seq = len(offsets) - 1
    n = lib().orc_build(residues, offsets, roles, n_seq, k, flags, None, None, 0)
    km = np.empty((n, k), np.uint8)
    rl = np.empty(n, np.int32)
    lib().orc_build(residues, offsets, roles, n_seq, k, flags, km.ctypes.data, rl.ctypes.data, n)
    return km, rl


def protein_distances(residues, offsets, pair_a, pair_b, k: int = 8, flags: int = 0):
    """SequenceKmers.distance per pair: (sim, |A|, |B|, distance) arrays."""
    pa = np.ascontiguousarray(pair_a, np.uint32)
    pb = np.ascontiguousarray(pair_b, np.uint32)
    n = len(pa)
    sim, sa, sb = np.empty(n, np.uint32), np.empty(n, np.uint32), np.empty(n, np.uint32)
    dist = np.empty(n, np.float64)
    lib().orc_protein_distances(residues, np.ascontiguousarray(offsets, np.uint64), k, flags,
                                pa, pb, n, sim, sa, sb, dist)
    return sim, sa, sb, dist



def propose(contig, left, strand, peg, peg_len, k: int = 8, min_strength: float = 0.5,
            max_fuzz: float = 1.5, min_fuzz: float = 0.8):
    """The projector's proposal sweep (KmerProcessor.java:209-264) over the connections
    (contig, left, strand, peg): (proposal arrays dict, stats[4])."""
    L = lib()
    if not getattr(L, "_propose_typed", False):
        L.orc_propose.restype = C.c_uint64
        L._propose_typed = True
    n = len(contig)
    args = [np.ascontiguousarray(contig, np.uint32), np.ascontiguousarray(left, np.int32),
            np.ascontiguousarray(strand, np.uint8), np.ascontiguousarray(peg, np.uint32)]
    pl = np.ascontiguousarray(peg_len, np.uint32)
    st = np.zeros(4, np.uint64)
    ptr = [a.ctypes.data_as(C.c_void_p) for a in args]
    cfg = [C.c_uint64(n), pl.ctypes.data_as(C.c_void_p), C.c_int(k), C.c_double(min_strength),
           C.c_double(max_fuzz), C.c_double(min_fuzz)]
    z = [None] * 7
    m = L.orc_propose(*ptr, *cfg, *z, C.c_uint64(0), st.ctypes.data_as(C.c_void_p))
    out = {"peg": np.empty(m, np.uint32), "contig": np.empty(m, np.uint32),
           "strand": np.empty(m, np.uint8), "left": np.empty(m, np.int32),
           "right": np.empty(m, np.int32), "evidence": np.empty(m, np.uint32),
           "frame": np.empty(m, np.uint8)}
    outs = [out[key].ctypes.data_as(C.c_void_p) for key in
            ("peg", "contig", "strand", "left", "right", "evidence", "frame")]
    L.orc_propose(*ptr, *cfg, *outs, C.c_uint64(m), st.ctypes.data_as(C.c_void_p))
    return out, st


def hash_annotate(gres, goff, pres, poff, k: int = 8, min_sim: float = 0.0125):
    """HashAnnotationProcessor's scoring loop: (best prototype per genome protein or -1,
    its similarity, matches per prototype)."""
    L = lib()
    n_gp, n_pt = len(goff) - 1, len(poff) - 1
    best = np.empty(n_gp, np.int32)
    sim = np.empty(n_gp, np.float64)
    cnt = np.empty(n_pt, np.uint32)
    vp = C.c_void_p
    L.orc_hash_annotate(np.ascontiguousarray(gres, np.uint8).ctypes.data_as(vp),
                        np.ascontiguousarray(goff, np.uint64).ctypes.data_as(vp), C.c_uint32(n_gp),
                        np.ascontiguousarray(pres, np.uint8).ctypes.data_as(vp),
                        np.ascontiguousarray(poff, np.uint64).ctypes.data_as(vp), C.c_uint32(n_pt),
                        C.c_int(k), C.c_double(min_sim), best.ctypes.data_as(vp),
                        sim.ctypes.data_as(vp), cnt.ctypes.data_as(vp))
    return best, sim, cnt
