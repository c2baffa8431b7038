#!/usr/bin/env python3
"""Interleaved A/B of the protein step in ONE process (workload and table built once): for each
workload, every option configuration is timed `reps` times in turn (device entry point, hipEvents
around `steps` calls), so that the arms share the box, the table and the batch. One JSON line per
(workload, config, rep) on stdout. The library is whatever KMERANNO_LIB names (an older build's
library compares kernels across commits: run the script once per library).

  python scripts/ab_protein.py [--workloads c5,c4,c2] [--configs packed=2;packed=0] [--reps 2]
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


def parse_config(text):
    out = {}
    for part in filter(None, text.split(",")):
        k, v = part.split("=")
        out[{"packed": "packed_input"}.get(k, k)] = int(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c5,c4,c2")
    ap.add_argument("--configs", default="packed=2;packed=0")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream().cuda_stream
    lib = os.environ.get("KMERANNO_LIB", "default")
    for wl in args.workloads.split(","):
        n_seq, t_size, n_fid, seed = synth.CONFIGS[wl]
        t0 = time.perf_counter()
        sig = synth.make_table(t_size, n_fid, seed, K)
        res, off, _, _ = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
        n_res = int(off[-1])
        n_win = int(np.maximum(np.diff(off).astype(np.int64) - K + 1, 0).sum())
        log(f"{wl}: generated in {time.perf_counter() - t0:.0f}s")
        table = kmeranno.SignatureTable.from_packed(sig.keys, sig.fids, K)
        ws = kmeranno.Workspace(0, n_res)
        d_res = torch.from_numpy(res).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        outs = [torch.empty(n_seq, dtype=d, device=dev) for d in (torch.int32, torch.int32, torch.uint8)]
        ref = None
        for rep in range(args.reps):
            for cfg_text in args.configs.split(";"):
                cfg = parse_config(cfg_text)
                with kmeranno.options(**cfg):
                    def call():
                        kmeranno.annotate_proteins_device(table, ws, d_res.data_ptr(),
                                                          d_off.data_ptr(), n_seq, n_res, 5, 0,
                                                          *[o.data_ptr() for o in outs], 0, 0, sp)
                    for _ in range(3):
                        call()
                    torch.cuda.synchronize()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(args.steps):
                        call()
                    b.record()
                    torch.cuda.synchronize()
                    ms = a.elapsed_time(b) / args.steps
                    ws.timing(True)
                    for _ in range(args.steps):
                        call()
                    n_t, ph = ws.phases_read()
                    ws.timing(False)
                got = tuple(o.cpu().numpy().copy() for o in outs)
                if ref is None:
                    ref = got
                same = all((x == y).all() for x, y in zip(got, ref))
                print(json.dumps({"workload": wl, "config": cfg_text, "rep": rep, "ms": ms,
                                  "phases_ms": {k: v / max(n_t, 1) for k, v in ph.items()},
                                  "lookups_per_s": n_win / (ms * 1e-3), "windows": n_win,
                                  "outputs_equal_first_arm": bool(same), "library": lib}),
                      flush=True)
        ws.close()
        table.close()
        del d_res, d_off, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
