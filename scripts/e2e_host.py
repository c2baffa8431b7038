#!/usr/bin/env python3
"""The c5 host call (kma_annotate_proteins: pack while staging, H2D in pieces under the previous
piece's kernel, D2H) under a sweep of KMA_OPT_HOST_PIECES x KMA_OPT_HOST_THREADS, one process,
interleaved; one JSON line per (config, rep) on stdout with the best-of-3 call time. Under
`rocprofv3 --kernel-trace --memory-copy-trace` (`--configs` one entry) the trace shows how the
copies and the piece kernels overlap.

  python scripts/e2e_host.py [--configs "pieces=8,threads=16;pieces=16,threads=16"] [--reps 2]
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
import torch  # noqa: E402,F401  (binds torch's libamdhip64 first)
import kmeranno  # noqa: E402
from kmeranno import synth  # noqa: E402

K, MIN_HITS = 8, 5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5")
    ap.add_argument("--configs", default="pieces=8,threads=16;pieces=16,threads=16;"
                    "pieces=4,threads=16;pieces=8,threads=8;pieces=16,threads=32")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--calls", type=int, default=3)
    args = ap.parse_args()
    n_seq, t_size, n_fid, seed = synth.CONFIGS[args.workload]
    t0 = time.perf_counter()
    sig = synth.make_table(t_size, n_fid, seed, K)
    res, off, _, _ = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
    print(f"generated in {time.perf_counter() - t0:.0f}s", file=sys.stderr, flush=True)
    table = kmeranno.SignatureTable.from_packed(sig.keys, sig.fids, K)
    names = {"pieces": "host_pieces", "threads": "host_threads", "packed": "packed_input"}
    lib = kmeranno.load()
    prof = (C.c_double * 6)()
    lib.kma_debug_host_profile.argtypes = [C.c_void_p, C.c_int]
    keys = ("setup", "stage", "launch", "wait", "outputs", "total")
    ref = None
    n = len(off) - 1
    # the caller's output arrays, reused across calls as bench.py's e2e_host does (fresh arrays
    # add their page faults and the previous ones' unmapping to every timed call)
    out = (np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.uint8),
           np.zeros(n_fid, np.uint32))
    for rep in range(args.reps):
        for text in args.configs.split(";"):
            cfg = {names[k]: int(v) for k, v in (p.split("=") for p in text.split(",") if p)}
            with kmeranno.options(**cfg):
                kmeranno.annotate_proteins(table, res, off, MIN_HITS, 0, n_fid=n_fid, out=out)
                best, best_prof = 1e30, None
                for _ in range(args.calls):
                    t1 = time.perf_counter()
                    got = kmeranno.annotate_proteins(table, res, off, MIN_HITS, 0, n_fid=n_fid,
                                                     out=out)
                    dt = time.perf_counter() - t1
                    if dt < best:
                        lib.kma_debug_host_profile(C.addressof(prof), 6)
                        best, best_prof = dt, dict(zip(keys, (round(x, 4) for x in prof)))
            got = tuple(a.copy() for a in got)
            if ref is None:
                ref = got
            same = all(np.array_equal(a, b) for a, b in zip(got, ref))
            print(json.dumps({"workload": args.workload, "config": text, "rep": rep,
                              "ms": best * 1e3, "residues": int(off[-1]),
                              "host_profile_ms": best_prof,
                              "outputs_equal_first": bool(same)}), flush=True)
    table.close()


if __name__ == "__main__":
    main()
