#!/usr/bin/env python3
"""Host-call staging experiment (measurement only): the library's pool packer
(kma_pack_residues, AVX2, non-temporal stores) writing c5's packed stream into pinned host
memory vs straight into fine-grained device memory through the PCIe BAR, each alone and each
beside a DMA of another pinned buffer (the pipeline's steady state: the link copies one segment
while the pool packs the next). Prints one JSON line of ms per case (best of --reps).

  python scripts/bar_mix_bench.py [--residues 310000000]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kmers.anno_amd", "python")]
import torch  # noqa: E402
import kmeranno  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--residues", type=int, default=310_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    n = args.residues
    kmeranno.load()
    lib = C.CDLL(kmeranno.LIB_PATH)  # raw pointers (the binding's argtypes take arrays)
    lib.kma_pack_residues.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64]
    hip = C.CDLL("libamdhip64.so")
    rng = np.random.default_rng(1)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    res = aa[rng.integers(0, 20, n + 64, dtype=np.uint8)]
    nbytes = kmeranno.packed_bytes(n)
    pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    pinned2 = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    bar = C.c_void_p()
    rc = hip.hipExtMallocWithFlags(C.byref(bar), C.c_size_t(nbytes), C.c_uint(1))  # fine-grained
    assert rc == 0, f"hipExtMallocWithFlags: {rc}"
    s = torch.cuda.Stream()

    def pack(dst_ptr, lo, hi):  # residues [lo, hi) -> the stream's bytes from group lo / 64
        rc = lib.kma_pack_residues(None, res[lo:].ctypes.data_as(C.c_void_p), hi - lo,
                                   C.c_void_p(dst_ptr + 40 * (lo // 64)),
                                   kmeranno.packed_bytes(hi - lo))
        assert rc == 0

    def dma(nb):
        with torch.cuda.stream(s):
            dev[:nb].copy_(pinned2[:nb], non_blocking=True)

    pack(bar.value, 0, n)  # first touch of the BAR mapping (slow once)
    out = {"residues": n, "packed_bytes": nbytes}

    def timed(name, fn):
        best = 1e30
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        out[name] = round(best * 1e3, 3)

    timed("pack_pinned", lambda: pack(pinned.data_ptr(), 0, n))
    timed("pack_bar", lambda: pack(bar.value, 0, n))
    timed("dma", lambda: dma(nbytes))
    timed("pack_pinned_with_dma", lambda: (dma(nbytes), pack(pinned.data_ptr(), 0, n)))
    timed("pack_bar_with_dma", lambda: (dma(nbytes), pack(bar.value, 0, n)))
    print(json.dumps(out), flush=True)
    hip.hipFree(bar)


if __name__ == "__main__":
    main()
