#!/usr/bin/env python3
"""Minimizer-layout robustness and per-genome latency (GPU box; one JSON line per case):

  sig_small_gto   signature table built by kma_build_signatures from small.gto's pegs (roles =
                  their functions): layout, displaced keys, longest chain; the protein path on
                  small.gto's pegs repeated to ~1M proteins (device entry point, hipEvent timed)
  adversarial     2.4M keys built to share 2,000 minimizers (every key holds one of the 2,000
                  6-mers lowest in the shipped m-mer order, so it is the key's minimizer): the
                  creators' choice (two-choice placement, rebuilt flat when crowded) vs the
                  forced m=7 layout, each timed on 200k proteins assembled from the keys
  per_genome      kma_annotate_proteins (host entry point: pinned staging, H2D, kernel, D2H on the
                  table's pooled stream) on ONE genome (small.gto's 712 pegs) against the 10^7-row
                  c2 table: the drop-in's per-genome call latency (median of 50)
"""
import gzip
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
dev = torch.device("cuda", 0)


def out(d):
    print(json.dumps(d), flush=True)


def info(t):
    i = t.info
    return {"entries": int(i.n_entries), "buckets": int(i.n_buckets), "layout_m": int(i.minimizer_len),
            "displaced": int(i.n_displaced), "displaced_frac": i.n_displaced / max(i.n_entries, 1),
            "longest_chain": int(i.max_probe), "two_choice": int(i.two_choice),
            "table_MiB": i.bytes / 2**20}


def time_device(t, res, off, reps=20):
    n = len(off) - 1
    n_res = int(off[-1] - off[0])
    ws = kmeranno.Workspace(0, n_res)
    d_res = torch.from_numpy(res).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    o = [torch.empty(n, dtype=x, device=dev) for x in (torch.int32, torch.int32, torch.uint8)]
    s = torch.cuda.current_stream().cuda_stream

    def call():
        kmeranno.annotate_proteins_device(t, ws, d_res.data_ptr(), d_off.data_ptr(), n, n_res, 5,
                                          0, *[x.data_ptr() for x in o], 0, 0, s)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        call()
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    wins = int(np.maximum(np.diff(off).astype(np.int64) - K + 1, 0).sum())
    st = o[2].cpu().numpy()
    ws.close()
    return {"proteins": n, "windows": wins, "ms": ms, "lookups_per_s": wins / (ms * 1e-3),
            "called": int((st == 1).sum())}


def repeat(res, off, times):
    lens = np.diff(off).astype(np.int64)
    allres = np.tile(res[:int(off[-1])], times)
    alloff = np.zeros(len(lens) * times + 1, np.uint64)
    alloff[1:] = np.cumsum(np.tile(lens, times))
    return np.concatenate([allres, np.zeros(64, np.uint8)]), alloff


def main():
    g = json.load(gzip.open(os.path.join(ROOT, "tests", "golden", "small.gto.gz"), "rt"))
    pegs = [f for f in g["features"] if f.get("protein_translation")]
    prots = [f["protein_translation"] for f in pegs]
    res, off = kmeranno.pack_strings(prots)
    # 1. signature table from small.gto (BuildKmerProcessor on the GPU)
    ids = {}
    roles = np.array([ids.setdefault(f.get("function", ""), len(ids)) for f in pegs], np.int32)
    keys, rl = kmeranno.build_signatures(res, off, roles, K)
    with kmeranno.SignatureTable.from_packed(keys, rl, K) as t:
        r2, o2 = repeat(res, off, 1400)
        out({"case": "sig_small_gto", "signature_keys": len(keys), "roles": len(ids), **info(t),
             **time_device(t, r2, o2)})
    # 2. adversarial keys sharing minimizers
    rng = np.random.default_rng(23)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)

    cand = aa[rng.integers(0, 20, (2_000_000, 6))]
    packed = np.zeros(len(cand), np.uint64)
    for j in range(6):
        packed = (packed << np.uint64(5)) | (cand[:, j].astype(np.uint64) - np.uint64(64))
    # the shipped m-mer order (kma_internal.h mmer_hash, KMA_HASH_LITE): one 32-bit multiply
    h = (packed * np.uint64(0x9E3779B1)) & np.uint64(0xFFFFFFFF)
    cores = cand[np.argsort(h)[:2000]]
    codes = np.arange(1, 21, dtype=np.uint64)[rng.integers(0, 20, (2000, 3, 400, 2))]
    keyset = set()
    for ci in range(2000):
        core = 0
        for j in range(6):
            core = (core << 5) | int(cores[ci, j] - 64)
        for pos in range(3):
            for x in range(400):
                a0, a1 = int(codes[ci, pos, x, 0]), int(codes[ci, pos, x, 1])
                # pos residues before the core, 2 - pos after (8 residues in all)
                pre = [a0, a1][:pos]
                suf = [a0, a1][pos:]
                v = 0
                for c in pre:
                    v = (v << 5) | c
                v = (v << 30) | core
                for c in suf:
                    v = (v << 5) | c
                keyset.add(v)
    akeys = np.array(sorted(keyset), np.uint64)
    afids = (np.arange(len(akeys)) % 5000).astype(np.uint32)
    letters = np.frombuffer(b"@ABCDEFGHIJKLMNOPQRSTUVWXYZ", np.uint8)
    pick = akeys[rng.integers(0, len(akeys), (200_000, 30))]
    byt = np.zeros((200_000, 30, 8), np.uint8)
    for j in range(8):
        byt[:, :, j] = letters[((pick >> np.uint64(5 * (7 - j))) & np.uint64(31)).astype(np.int64)]
    ares = np.concatenate([byt.reshape(-1), np.zeros(64, np.uint8)])
    aoff = (np.arange(200_001, dtype=np.uint64) * 240)
    for lf, forced in ((0.5, None), (0.9, None), (0.5, 6), (0.5, 7)):
        with kmeranno.options(**({"layout": forced} if forced else {})):
            t = kmeranno.SignatureTable.from_packed(akeys, afids, K, load_factor=lf)
        with t:
            out({"case": "adversarial", "load_factor": lf, "forced_layout": forced,
                 "keys": len(akeys), **info(t), **time_device(t, ares, aoff)})
    # 3. per-genome host-entry latency against the c2 table
    n_seq, t_size, n_fid, seed = synth.CONFIGS["c2"]
    sig = synth.make_table(t_size, n_fid, seed, K)
    with kmeranno.SignatureTable.from_packed(sig.keys, sig.fids, K) as t:
        for _ in range(3):
            kmeranno.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
        lat = []
        for _ in range(50):
            t0 = time.perf_counter()
            kmeranno.annotate_proteins(t, res, off, 5, 0, n_fid=n_fid)
            lat.append((time.perf_counter() - t0) * 1e3)
        out({"case": "per_genome", "entry": "kma_annotate_proteins (host buffers)",
             "genome": g["id"], "pegs": len(prots), "residues": int(off[-1]),
             "table_rows": t_size, "median_ms": float(np.median(lat)),
             "p90_ms": float(np.percentile(lat, 90))})


if __name__ == "__main__":
    main()
