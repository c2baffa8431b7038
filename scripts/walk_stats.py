#!/usr/bin/env python3
"""Chain-walk event counts of one protein launch (tuning only).

Needs a library built with the counters:
    make -C kmers.anno_amd variant VNAME=count VFLAGS=-DKMA_TUNE_COUNT
    KMERANNO_LIB=kmers.anno_amd/build/count/libkmeranno.so python scripts/walk_stats.py c5 [lf]

Prints one JSON line: flushes, queued walks, probed windows, home hits and walk hits of one
annotate_kernel launch over the workload, with the table's build statistics.
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402
from bench import K, MIN_HITS, kmeranno, synth  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
    lf = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    sp = torch.cuda.current_stream().cuda_stream
    n_seq, t_size, n_fid, seed = synth.CONFIGS[wl]
    sig = synth.make_table(t_size, n_fid, seed, K)
    residues, offsets, _, _ = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
    table, _ = bench.build_table(sig.keys, sig.fids, t_size, lf, dev, sp, 0, 1)
    n_res = int(offsets[-1] - offsets[0])
    ws = kmeranno.Workspace(0, n_res)
    d_res = torch.from_numpy(residues).to(dev)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    outs = [torch.empty(n_seq, dtype=d, device=dev) for d in (torch.int32, torch.int32, torch.uint8)]
    lib = C.CDLL(os.environ["KMERANNO_LIB"])
    st = np.zeros(8, np.uint64)
    assert lib.kma_debug_walk_stats(st.ctypes.data_as(C.c_void_p), 1) == 0
    kmeranno.annotate_proteins_device(table, ws, d_res.data_ptr(), d_off.data_ptr(), n_seq, n_res,
                                      MIN_HITS, 0, *[o.data_ptr() for o in outs], 0, 0, sp)
    torch.cuda.synchronize()
    assert lib.kma_debug_walk_stats(st.ctypes.data_as(C.c_void_p), 1) == 0
    n_win = int(np.maximum(np.diff(offsets).astype(np.int64) - K + 1, 0).sum())
    names = ["flushes", "queued_walks", "probed_windows", "home_hits", "walk_hits", "walk_hits_step1",
             "walk_buckets", "flush_longest_sum"]
    out = {"workload": wl, "load_factor": lf, "windows": n_win, "table": table.stats()
           if hasattr(table, "stats") else None}
    out.update({n: int(st[i]) for i, n in enumerate(names)})
    out["walks_per_probed"] = out["queued_walks"] / max(out["probed_windows"], 1)
    out["walk_hit_frac"] = out["walk_hits"] / max(out["queued_walks"], 1)
    out["walks_per_flush"] = out["queued_walks"] / max(out["flushes"], 1)
    out["buckets_per_walk"] = out["walk_buckets"] / max(out["queued_walks"], 1)
    out["walk_buckets_per_probed"] = out["walk_buckets"] / max(out["probed_windows"], 1)
    out["longest_per_flush"] = out["flush_longest_sum"] / max(out["flushes"], 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
