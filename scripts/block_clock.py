"""Per-block timeline of annotate_kernel (tuning only).

Needs a library built with the block clock:
    make -C kmers.anno_amd variant VNAME=clk VFLAGS=-DKMA_BLOCK_CLOCK
    KMERANNO_LIB=kmers.anno_amd/build/clk/libkmeranno.so python scripts/block_clock.py c2

Prints the kernel span, the block-duration distribution against each block's residue span, the
number of blocks resident over time and when the tail starts.
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


def contigs_timeline():
    """c3: contigs_probe_quad_kernel's blocks (256 x KMA_CONTIG_SEQ positions each): clock 0 start,
    1 tile loaded + contigs found, 2 translated, 3 bucket loads issued (last slice), 4 matched
    (last slice), 5 end (records staged, block count added)."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    sp = torch.cuda.current_stream().cuda_stream
    wl = synth.make_contig_workload(5_000_000, 20, 3, 10_000_000, 10_000, K)
    n_bases = int(wl.offsets[-1] - wl.offsets[0])
    table, _ = bench.build_table(wl.keys, wl.fids, 10_000_000, 0.5, dev, sp, 0, 1)
    ws = kmeranno.Workspace(0)
    ws.reserve_contigs(n_bases)
    d_dna = torch.from_numpy(wl.dna).to(dev)
    d_off = torch.from_numpy(wl.offsets.view(np.int64)).to(dev)
    cap = 1 << 22
    d_hits = torch.empty(cap * kmeranno.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_nh = torch.zeros(1, dtype=torch.int64, device=dev)
    for _ in range(5):
        kmeranno.annotate_contigs_device(table, ws, d_dna.data_ptr(), d_off.data_ptr(),
                                         len(wl.offsets) - 1, n_bases, 11, d_hits.data_ptr(), cap,
                                         d_nh.data_ptr(), 0, 0, sp)
    torch.cuda.synchronize()
    lib = C.CDLL(os.environ["KMERANNO_LIB"])
    full = np.zeros(8 * 65536, np.uint64)
    assert lib.kma_debug_block_clock(full.ctypes.data_as(C.c_void_p), C.c_uint64(8 * 65536)) == 0
    rows = full.reshape(65536, 8)
    nb = int((rows[:, 0] != 0).sum())  # blocks of the last launch (tile size from the build)
    clk = rows[:nb][:, :6].astype(np.int64)
    us = (clk - clk[:, 0].min()) * 10.0 / 1e3
    ph = np.diff(us, axis=1)
    names = ["tile_and_contigs", "translate", "slices_issue", "match", "compact_store"]
    s, e = us[:, 0], us[:, 5]
    grid = np.linspace(0, e.max(), 41)
    return {"workload": "c3", "blocks": int(nb), "kernel_span_us": float(e.max()),
            "last_start_us": float(s.max()),
            "dur_us_pct": {q: float(np.percentile(e - s, q)) for q in (5, 50, 95, 100)},
            "phase_us_median": {n: float(np.median(ph[:, i])) for i, n in enumerate(names)},
            "phase_us_p95": {n: float(np.percentile(ph[:, i], 95)) for i, n in enumerate(names)},
            "resident": [int(((s <= g) & (e > g)).sum()) for g in grid]}


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    if wl == "c3":
        print(json.dumps(contigs_timeline()))
        return
    bp = int(os.environ.get("KMA_BLOCK_PROTEINS", "4"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    sp = torch.cuda.current_stream().cuda_stream
    n_seq, t_size, n_fid, seed = synth.CONFIGS[wl]
    sig = synth.make_table(t_size, n_fid, seed, K)
    residues, offsets, _, _ = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
    if os.environ.get("ORDER") == "lpt":  # experiment: the same groups, longest span first
        lens = np.diff(offsets).astype(np.int64)
        gs = np.arange(0, n_seq, bp)
        order = np.argsort(-np.add.reduceat(lens, gs), kind="stable")
        perm = np.concatenate([np.arange(gs[g], min(gs[g] + bp, n_seq)) for g in order])
        residues = np.concatenate([residues[offsets[i]:offsets[i + 1]] for i in perm])
        offsets = np.concatenate([[0], np.cumsum(lens[perm])]).astype(offsets.dtype)
    table, _ = bench.build_table(sig.keys, sig.fids, t_size, 0.5, dev, sp, 0, 1)
    n_res = int(offsets[-1] - offsets[0])
    ws = kmeranno.Workspace(0, n_res)
    d_res = torch.from_numpy(residues).to(dev)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    d_fid = torch.empty(n_seq, dtype=torch.int32, device=dev)
    d_cnt = torch.empty(n_seq, dtype=torch.int32, device=dev)
    d_st = torch.empty(n_seq, dtype=torch.uint8, device=dev)
    for _ in range(5):
        kmeranno.annotate_proteins_device(table, ws, d_res.data_ptr(), d_off.data_ptr(), n_seq,
                                          n_res, MIN_HITS, 0, d_fid.data_ptr(), d_cnt.data_ptr(),
                                          d_st.data_ptr(), 0, 0, sp)
    torch.cuda.synchronize()
    lib = C.CDLL(os.environ["KMERANNO_LIB"])
    n_groups = (n_seq + bp - 1) // bp
    slots = 7 * torch.cuda.get_device_properties(0).multi_processor_count
    dv = os.environ.get("KMA_DEFER", "")
    two_pass = (int(dv) > 0) if dv else slots < n_groups <= 4 * slots  # kma_abi.cpp defer_below
    nb = min(2 * n_groups if two_pass else n_groups, 65535)
    full = np.zeros(8 * 65536, np.uint64)
    assert lib.kma_debug_block_clock(full.ctypes.data_as(C.c_void_p), C.c_uint64(8 * 65536)) == 0
    c = full[:8 * nb].reshape(nb, 8)
    clk = c[:, :6].astype(np.int64)
    base = clk[:, 0].min()
    work = clk[:, 1] > 0  # blocks that annotated a group (two-pass: the others exited early)
    us = (clk - base) * 10.0 / 1e3  # wall_clock64: 100 MHz
    s, e = us[:, 0], us[:, 5]
    w = us[work]
    steps = c[work, 7].astype(np.int64)
    dur = w[:, 5] - w[:, 0]
    ph = np.diff(w, axis=1)  # records, first step, other steps, chain walks, vote
    names = ["records", "first_step", "other_steps", "chain_walks", "vote"]
    out = {"workload": wl, "block_proteins": bp, "two_pass": bool(two_pass),
           "order": os.environ.get("ORDER"),
           "blocks": int(nb), "working_blocks": int(work.sum()),
           "kernel_span_us": float(e.max()), "last_work_start_us": float(w[:, 0].max()),
           "skipped_block_us_median": float(np.median((e - s)[~work])) if (~work).any() else None,
           "dur_us_pct": {q: float(np.percentile(dur, q)) for q in (5, 25, 50, 75, 95, 100)},
           "phase_us_median": {n: float(np.median(ph[:, i])) for i, n in enumerate(names)},
           "phase_us_p95": {n: float(np.percentile(ph[:, i], 95)) for i, n in enumerate(names)}}
    m = steps > 1
    if m.any():
        out["per_later_step_us_median"] = float(np.median(ph[m, 2] / (steps[m] - 1)))
    for st in sorted(set(steps.tolist()))[:10]:
        mm = steps == st
        out.setdefault("dur_by_steps", {})[int(st)] = [int(mm.sum()), float(np.median(dur[mm]))]
    grid = np.linspace(0, e.max(), 41)
    out["resident_working"] = [int(((w[:, 0] <= g) & (w[:, 5] > g)).sum()) for g in grid]
    xcc = (c[work, 6] >> np.uint64(32)).astype(np.int64)
    out["xcc_end_us"] = [float(w[xcc == x, 5].max()) if (xcc == x).any() else 0.0
                         for x in range(8)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
