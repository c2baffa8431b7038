"""CPU rehearsal of bench.py's multi-rank branch (test infrastructure, no GPU).

Run under torch.distributed.run with --dist-backend gloo: bench.main() runs unchanged, with
  - torch.cuda replaced by a host stand-in (events on the wall clock, no-op synchronize,
    devices mapped to the CPU), so device tensors are host tensors;
  - libkmeranno.so replaced by StubKmerAnno: the entry points bench.py calls, computed on the
    host with the same semantics (last-wins table in the slot array the broadcast moves,
    distinct-kmer sets, the vote) — the oracle's restatement, vectorized with numpy.
Python slips in the world > 1 branch (a lost global, a wrong keyword, a shape error in the
collectives or the report) then fail here instead of on the GPU box. Numbers are meaningless;
the JSON line's structure and the --verify checks are what the test reads.

  python -m torch.distributed.run --nproc-per-node 2 ... tests/bench_rehearsal.py <bench args>
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kmers.anno_amd", "python")]
from kmeranno import synth  # noqa: E402

K = 8
FID_BITS = 22


def _arr(ptr: int, n: int, dtype) -> np.ndarray:
    dt = np.dtype(dtype)
    if n == 0:
        return np.zeros(0, dt)
    buf = (C.c_uint8 * (n * dt.itemsize)).from_address(ptr)
    return np.frombuffer(buf, dt, n)


# ---- torch.cuda stand-in ------------------------------------------------------------------------
class _Event:
    def __init__(self, enable_timing=False):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3

    def synchronize(self):
        pass


class _Stream:
    cuda_stream = 0

    def __init__(self, device=None):
        pass


class _Props:
    name = "host stand-in"
    pci_bus_id = None


def _fake_cuda():
    m = types.SimpleNamespace()
    m.Event = _Event
    m.Stream = _Stream
    m.synchronize = lambda *a, **k: None
    m.set_device = lambda *a, **k: None
    m.current_stream = lambda *a, **k: _Stream()
    m.is_available = lambda: True
    m.get_device_properties = lambda *a, **k: _Props()
    m.stream = lambda s: _NullCtx()
    return m


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class _Device:
    """torch.device("cuda", i) for the rehearsal: the CPU, keeping the index bench.py reads."""

    def __new__(cls, kind, index=None):
        return torch.device("cpu")


class FakeTorch(types.ModuleType):
    def __init__(self):
        super().__init__("torch")
        self.cuda = _fake_cuda()
        self.device = _Device

    def __getattr__(self, name):
        return getattr(torch, name)


# ---- libkmeranno stand-in -----------------------------------------------------------------------
def _windows(res: np.ndarray, off: np.ndarray, s: int) -> np.ndarray:
    a, b = int(off[s]), int(off[s + 1])
    return np.unique(synth.window_keys(res[a:b], K))


def _vote(keys_sorted, fids_sorted, res, off, n_seq, min_hits):
    fid = np.full(n_seq, -1, np.int32)
    cnt = np.zeros(n_seq, np.int32)
    st = np.zeros(n_seq, np.uint8)
    for s in range(n_seq):
        w = _windows(res, off, s)
        if len(w) == 0 or len(keys_sorted) == 0:
            continue
        i = np.searchsorted(keys_sorted, w)
        i = np.minimum(i, len(keys_sorted) - 1)
        hit = keys_sorted[i] == w
        if not hit.any():
            continue
        f = fids_sorted[i[hit]]
        if f.min() != f.max():
            st[s] = 2
            continue
        fid[s], cnt[s] = int(f[0]), int(hit.sum())
        st[s] = 1 if cnt[s] >= min_hits else 3
    return fid, cnt, st


class _Info:
    def __init__(self, nb, device, m):
        self.n_buckets = nb
        self.bytes = nb * 8 * 8
        self.device = 0 if device is None else device
        self.minimizer_len = m & 0x3F
        self.minimizer_order = 1 if m & 0x40 else 0
        self.two_choice = 1 if m & 0x100 else 0
        self.k = K


class _Table:
    def __init__(self, ptr, nb, device, m):
        self.ptr, self.nb = ptr, nb
        self.info = _Info(nb, device, m)
        self.replicas = [self.info.device]

    def contents(self):
        s = _arr(self.ptr, self.nb * 8, np.uint64)
        s = s[s != 0]
        return s >> np.uint64(FID_BITS), (s & np.uint64((1 << FID_BITS) - 1)).astype(np.int32)

    def replicate(self, devices):
        self.replicas = self.replicas + list(devices)

    def close(self):
        pass


class _Workspace:
    def __init__(self, device=0, n_residues=0, n_seq=0):
        self.on, self.calls = False, 0

    def timing(self, enable=True):
        self.on, self.calls = enable, 0

    def phases_read(self):
        n, self.calls = self.calls, 0
        return n, {"annotate_kernel": 1.0 * n}

    def reserve_contigs(self, n):
        pass

    def close(self):
        pass


class StubKmerAnno(types.ModuleType):
    STATUS_CALLED = 1
    OPT_PACKED_INPUT = 6
    OPT_PLACEMENT = 9
    LAYOUT_TWO_CHOICE = 0x100
    LAYOUT_MOD_SAMPLING = 0x40
    HIT_DTYPE = np.dtype([("contig", "<u4"), ("left", "<i4"), ("fid", "<u4"), ("strand", "u1"),
                          ("frame", "u1"), ("pad", "<u2")])

    def __init__(self):
        super().__init__("kmeranno")
        self._opts = {6: 1}
        self.SignatureTable = types.SimpleNamespace(
            wrap_device=lambda ptr, nb, k, device, m: _Table(ptr, nb, device, m))
        self.Workspace = _Workspace

    def set_option(self, o, v):
        self._opts[o] = v

    def get_option(self, o):
        return self._opts.get(o, 0)

    def options(self, **kw):
        return _NullCtx()

    def source_digest(self):
        return "stub"

    def buckets_for(self, n, lf=0.5, k=8):
        return max(1, int(np.ceil(n / lf / 8)))

    def bucket_slots(self, k=8):
        return 8

    def choose_layout(self, k, nb, build):
        return 6 | 0x100, build(6 | 0x100)

    def build_device(self, d_slots, nb, d_winner, d_keys, d_fids, n, d_status, stream, k=8,
                     layout=-1):
        keys = _arr(d_keys, n, np.uint64)
        fids = _arr(d_fids, n, np.uint32)
        last = {}
        for key, f in zip(keys.tolist(), fids.tolist()):  # HashMap.put: the last row wins
            if key and key >> (5 * k) == 0:
                last[key] = f
        ks = np.array(sorted(last), np.uint64)
        slots = _arr(d_slots, nb * 8, np.uint64)
        slots[:] = 0
        slots[:len(ks)] = (ks << np.uint64(FID_BITS)) | np.array([last[x] for x in ks.tolist()],
                                                                 np.uint64)
        _arr(d_status, 4, np.int32)[:] = [0, len(ks), 1, 0]

    def annotate_proteins_device(self, table, ws, d_res, d_off, n_seq, n_res, min_hits, flags,
                                 d_fid, d_cnt, d_st, d_tally, n_fid, stream):
        off = _arr(d_off, n_seq + 1, np.uint64)
        res = _arr(d_res, int(off[-1]) + 32, np.uint8)
        keys, fids = table.contents()
        fid, cnt, st = _vote(keys, fids, res, off, n_seq, min_hits)
        _arr(d_fid, n_seq, np.int32)[:] = fid
        _arr(d_cnt, n_seq, np.int32)[:] = cnt
        _arr(d_st, n_seq, np.uint8)[:] = st
        if d_tally:
            t = _arr(d_tally, n_fid, np.int32)
            np.add.at(t, fid[(st == 1) & (fid < n_fid)], 1)
        ws.calls += ws.on

    def annotate_proteins(self, table, residues, offsets, min_hits, flags, n_fid=None):
        keys, fids = table.contents()
        n_seq = len(offsets) - 1
        fid, cnt, st = _vote(keys, fids, residues, np.asarray(offsets, np.uint64), n_seq,
                             min_hits)
        if n_fid is None:
            return fid, cnt, st
        return fid, cnt, st, np.bincount(fid[st == 1], minlength=n_fid).astype(np.uint32)


def main():
    import bench
    bench.torch = FakeTorch()
    bench.kmeranno = StubKmerAnno()
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()


if __name__ == "__main__":
    main()
