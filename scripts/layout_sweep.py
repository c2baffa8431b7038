#!/usr/bin/env python3
"""c5 table-layout sweep on the GPU box (one JSON line per case, stdout).

The c5 batch (1M proteins, BASELINE configs[4]) is generated once; for every load factor and
every layout (minimizer m = 6, m = 7, flat) the 10^8-row table is built on the device with the
layout forced (kma_table_build_device), its build statistics recorded (displaced keys, longest
chain), and the protein path timed over the batch (device entry point, hipEvents on the
stream). "auto" marks the layout the library's creators would keep at that size and load
factor (kmeranno.choose_layout = kma_abi.cpp create_from_device_keys: the size rule, then an
m = 7 rebuild of a table with > 10% displaced keys, then a flat one of a crowded table).

Dispatch order is deterministic (cases in the printed order, each `warmup + steps`
annotate_kernel launches), so a rocprofv3 --pmc run of this script attributes counters per case
(scripts/sweep_pmc_summary.py).

  python scripts/layout_sweep.py [--lfs 0.5,0.75,0.9] [--layouts 6,7,0] [--steps 10]
         [--n-seq 1000000] [--adversarial]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kmers.anno_amd", "python")]
import kmeranno  # noqa: E402
from kmeranno import synth  # noqa: E402

K = 8


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lfs", default="0.5,0.75,0.9")
    ap.add_argument("--layouts", default="6,7,0")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n-seq", type=int, default=0)
    ap.add_argument("--adversarial", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream().cuda_stream
    n_seq, t_size, n_fid, seed = synth.CONFIGS["c5"]
    n_seq = args.n_seq or n_seq
    t0 = time.perf_counter()
    if args.adversarial:
        keys, fids, res, off = adversarial_workload()
        t_size = len(keys)
    else:
        sig = synth.make_table(t_size, n_fid, seed, K)
        res, off, _, _ = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
        keys, fids = sig.keys, sig.fids
    n_seq = len(off) - 1
    n_res = int(off[-1] - off[0])
    n_win = int(np.maximum(np.diff(off).astype(np.int64) - K + 1, 0).sum())
    log(f"workload: {len(keys)} rows, {n_seq} proteins, {n_win} windows "
        f"({time.perf_counter() - t0:.0f}s)")
    d_keys = torch.from_numpy(keys.view(np.int64)).to(dev)
    d_fids = torch.from_numpy(fids.view(np.int32)).to(dev)
    d_res = torch.from_numpy(res).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    outs = [torch.empty(n_seq, dtype=d, device=dev) for d in (torch.int32, torch.int32, torch.uint8)]
    ws = kmeranno.Workspace(0, n_res)
    status = torch.zeros(4, dtype=torch.int32, device=dev)
    ref = None
    for lf in [float(x) for x in args.lfs.split(",")]:
        nb = kmeranno.buckets_for(t_size, lf)
        slots = torch.empty(nb * kmeranno.bucket_slots(), dtype=torch.int64, device=dev)
        winner = torch.empty(nb * kmeranno.bucket_slots(), dtype=torch.int32, device=dev)
        stats = {}
        for m in [int(x) for x in args.layouts.split(",")]:
            kmeranno.build_device(slots.data_ptr(), nb, winner.data_ptr(), d_keys.data_ptr(),
                                  d_fids.data_ptr(), len(keys), status.data_ptr(), sp, k=K,
                                  layout=m)
            torch.cuda.synchronize()
            st = status.cpu().numpy().astype(np.int64)
            if st[0]:  # report and go on (a table-full build answers wrongly: not timed)
                print(json.dumps({"case": "table_full", "load_factor": lf, "layout_m": m,
                                  "status": st.tolist()}), flush=True)
                continue
            t = kmeranno.SignatureTable.wrap_device(slots.data_ptr(), nb, K, 0, m)

            def call():
                kmeranno.annotate_proteins_device(t, ws, d_res.data_ptr(), d_off.data_ptr(),
                                                  n_seq, n_res, 5, 0,
                                                  *[o.data_ptr() for o in outs], 0, 0, sp)
            for _ in range(args.warmup):
                call()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.steps):
                call()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.steps
            got = tuple(o.cpu().numpy().copy() for o in outs)
            if ref is None:
                ref = got
            same = all((x == y).all() for x, y in zip(got, ref))
            t.close()
            stats[m] = st
            rec = {"case": "adversarial" if args.adversarial else "c5", "load_factor": lf,
                   "layout_m": m, "buckets": nb, "entries": int(st[1]),
                   "longest_chain": int(st[2]), "displaced": int(st[3]),
                   "displaced_frac": st[3] / max(st[1], 1), "ms": ms,
                   "lookups_per_s": n_win / (ms * 1e-3), "windows": n_win,
                   "launches": args.warmup + args.steps, "outputs_equal_first_case": bool(same),
                   "library": os.environ.get("KMERANNO_LIB", "default")}
            print(json.dumps(rec), flush=True)
        # which layout the creators keep (kma_abi.cpp create_from_device_keys)
        msize = kmeranno.layout_for(K, nb)
        if set(stats) >= {0, 6, 7}:
            pick, _ = kmeranno.choose_layout(K, nb, lambda m: stats[m])
            print(json.dumps({"case": "auto", "load_factor": lf, "size_rule_m": msize,
                              "creator_keeps_m": pick}), flush=True)
        del slots, winner
        torch.cuda.empty_cache()
    ws.close()


def adversarial_workload():
    """~1.5M keys built to share 2,000 minimizers and 200k proteins assembled from them: the
    cores are the 2,000 6-mers of lowest m-mer hash (kma_internal.h mmer_hash, KMA_HASH_LITE:
    the 32-bit product with 0x9E3779B1) among 2M random ones, so every key built around one has
    it as its minimizer at m = 6."""
    rng = np.random.default_rng(23)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    cand = aa[rng.integers(0, 20, (2_000_000, 6))]
    packed = np.zeros(len(cand), np.uint64)
    for j in range(6):
        packed = (packed << np.uint64(5)) | (cand[:, j].astype(np.uint64) - np.uint64(64))
    h = (packed * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)
    cores = packed[np.argsort(h)[:2000]]
    codes = np.arange(1, 21, dtype=np.uint64)[rng.integers(0, 20, (2000, 3, 400, 2))]
    ks = []
    for pos in range(3):
        a0, a1 = codes[:, pos, :, 0], codes[:, pos, :, 1]
        core = cores[:, None]
        if pos == 0:
            v = (core << np.uint64(10)) | (a0 << np.uint64(5)) | a1
        elif pos == 1:
            v = (a0 << np.uint64(35)) | (core << np.uint64(5)) | a1
        else:
            v = (a0 << np.uint64(35)) | (a1 << np.uint64(30)) | core
        ks.append(v.reshape(-1))
    keys = np.unique(np.concatenate(ks))
    fids = (np.arange(len(keys)) % 5000).astype(np.uint32)
    letters = np.frombuffer(b"@ABCDEFGHIJKLMNOPQRSTUVWXYZ", np.uint8)
    pick = keys[rng.integers(0, len(keys), (200_000, 30))]
    byt = np.zeros((200_000, 30, 8), np.uint8)
    for j in range(8):
        byt[:, :, j] = letters[((pick >> np.uint64(5 * (7 - j))) & np.uint64(31)).astype(np.int64)]
    res = np.concatenate([byt.reshape(-1), np.zeros(64, np.uint8)])
    off = np.arange(200_001, dtype=np.uint64) * 240
    return keys, fids, res, off


if __name__ == "__main__":
    main()
