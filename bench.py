#!/usr/bin/env python3
"""Benchmark of the signature-kmer annotation hot path on MI355X (BASELINE.json metric).

One step = one annotate pass (ProteinKmers extraction + table probe + vote, the loop of
ApplyKmerProcessor.java:122-147) over one rank's batch of synthetic proteins already resident
in HBM, through the C ABI's device entry point (libkmeranno.so). The per-function tallies of
the APPLY report accumulate on device across steps and are reduced to rank 0 over RCCL once,
inside the timed region (the only exchange step of the path). Scaling is weak: every rank
annotates its own batch against its replica of the table (built on rank 0, broadcast).

With --workload c3 one step is one 6-frame pass (KmerReference.java:157-203: translate both
strands in three frames, skip '*'/'X' windows, probe the table, emit hits in canonical order)
over a rank's resident synthetic genome (kma_annotate_contigs_device).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c5]
  torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch  # first: libkmeranno.so must bind torch's libamdhip64 (same SONAME)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kmers.anno_amd", "python")]
import kmeranno  # noqa: E402
from kmeranno import dist as kdist  # noqa: E402
from kmeranno import synth  # noqa: E402

K = 8
MIN_HITS = 5
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec
BYTES_PER_LOOKUP = 64  # one 64-byte bucket line per probe
# kma_gather_bench, 1.5 GiB buffer, quad shape (profiles/r01_gather_bench.jsonl): random 64-B
# lines beyond L2 are served at ~5.5e10/s on MI355X.
GATHER_CEILING_GBS = 3544.2
# Per-launch HBM traffic of K1 from rocprofv3 FETCH_SIZE + WRITE_SIZE passes (scripts/
# gpu_traffic.sh), calibrated on the gather bench (scripts/traffic_summary.py).
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r01c_traffic.json")
WORKLOADS = {
    "c2": "10k synthetic proteins (small.gto CDS length distribution) vs 10M-entry protein "
          "8-mer signature table, 1 MI355X per rank",
    "c3": "whole-contig 6-frame DNA->protein kmer annotation: 5 Mbp synthetic genome per rank "
          "(20 contigs, log-uniform 50 kb-1 Mbp, GC 0.5, 0.05% n, genes planted on both strands "
          "over ~50%, code 11) vs 10M-entry protein 8-mer table",
    "c4": "1M-protein metagenome batch per rank vs 10M-entry table (replicated)",
    "c5": "1M proteins per rank vs 10^8-entry multi-function signature table "
          "(HBM random access)",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(sig, residues, offsets, budget_s=10.0):
    """The C oracle (scalar restatement of ApplyKmerProcessor's table load + loop: chained
    String hash map + per-protein kmer set) timed on one host core over a bounded sample."""
    from oracle import c_oracle
    c_oracle.build()
    n = len(sig.keys)
    kmers = np.zeros((n, K), np.uint8)
    for j in range(K):
        kmers[:, j] = ((sig.keys >> np.uint64(5 * (K - 1 - j))) & np.uint64(31)).astype(np.uint8) + 64
    t0 = time.perf_counter()
    table = c_oracle.Table.from_buffer(kmers.tobytes(), np.arange(n + 1, dtype=np.uint64) * K,
                                       sig.fids.astype(np.int32))
    load_s = time.perf_counter() - t0
    lens = np.diff(offsets).astype(np.int64)
    n_seq, lookups, reps = len(lens), 0, 0
    # sample: leading proteins of the batch, doubled until the sample takes >= budget/4
    take = min(n_seq, 500)
    while True:
        sub_off = offsets[:take + 1].copy()
        t0 = time.perf_counter()
        c_oracle.apply(table, residues, sub_off, K, MIN_HITS, 0)
        dt = time.perf_counter() - t0
        if dt >= budget_s / 4 or take == n_seq:
            break
        take = min(n_seq, take * 2)
    wins = int(np.maximum(lens[:take] - K + 1, 0).sum())
    total_t, reps = 0.0, 0
    while total_t < budget_s and reps < 20:
        t0 = time.perf_counter()
        c_oracle.apply(table, residues, sub_off, K, MIN_HITS, 0)
        total_t += time.perf_counter() - t0
        reps += 1
        lookups += wins
    return {"value": lookups / total_t, "unit": "kmer lookups/s", "cores": 1, "kind": "port",
            "sample": f"oracle/kma_oracle.c orc_apply on the first {take} proteins of the rank-0 "
                      f"batch ({wins} windows) x {reps} reps against the same {n}-entry table "
                      f"(table load {load_s:.1f}s, untimed)"}


def cpu_baseline_contigs(wl, budget_s=10.0):
    """The C oracle's 6-frame pass (translate + processKmers window filter + String-keyed map
    probe per window, KmerReference.java:157-203) on one host core, over leading contigs."""
    from oracle import c_oracle
    c_oracle.build()
    n = len(wl.keys)
    kmers = np.zeros((n, K), np.uint8)
    for j in range(K):
        kmers[:, j] = ((wl.keys >> np.uint64(5 * (K - 1 - j))) & np.uint64(31)).astype(np.uint8) + 64
    t0 = time.perf_counter()
    table = c_oracle.Table.from_buffer(kmers.tobytes(), np.arange(n + 1, dtype=np.uint64) * K,
                                       wl.fids.astype(np.int32))
    load_s = time.perf_counter() - t0
    take, total_t, wins, reps = 1, 0.0, 0, 0
    while total_t < budget_s and reps < 50:
        off = wl.offsets[:take + 1].copy()
        t0 = time.perf_counter()
        c_oracle.annotate_contigs(table, wl.dna, off, 11, K)
        dt = time.perf_counter() - t0
        total_t += dt
        reps += 1
        wins += kmeranno.contig_window_count(off, K)
        if dt < budget_s / 8 and take < wl.n_contig:
            take += 1
    return {"value": wins / total_t, "unit": "kmer lookups/s", "cores": 1, "kind": "port",
            "sample": f"oracle/kma_oracle.c orc_annotate_contigs on leading contigs of the rank-0 "
                      f"genome (1..{take} contigs per rep, {reps} reps, {wins} 6-frame windows) "
                      f"against the same {n}-entry table (table load {load_s:.1f}s, untimed)"}


def build_table(keys_np, fids_np, t_size, load_factor, dev, sp, rank, world):
    """Signature table built on rank 0's GPU, replicated over RCCL (xGMI) to the other ranks."""
    nb = kmeranno.buckets_for(t_size, load_factor)
    slots = torch.empty(nb * 8, dtype=torch.int64, device=dev)
    if rank == 0:
        winner = torch.empty(nb * 8, dtype=torch.int32, device=dev)
        status = torch.zeros(4, dtype=torch.int32, device=dev)
        keys = torch.from_numpy(keys_np.view(np.int64)).to(dev)
        fids = torch.from_numpy(fids_np.view(np.int32)).to(dev)
        tb = torch.cuda.Event(enable_timing=True)
        te = torch.cuda.Event(enable_timing=True)
        tb.record()
        kmeranno.build_device(slots.data_ptr(), nb, winner.data_ptr(), keys.data_ptr(),
                              fids.data_ptr(), t_size, status.data_ptr(), sp, k=K)
        te.record()
        torch.cuda.synchronize()
        st = status.cpu().numpy()
        assert st[0] == 0, "table full"
        log(f"[rank 0] table: {st[1]} entries, {nb} buckets ({nb * 64 / 2**20:.0f} MiB), "
            f"max probe {st[2]}, built in {tb.elapsed_time(te):.1f} ms")
        del winner, keys, fids
    if world > 1:
        kdist.broadcast_table(slots, src=0)  # RCCL over xGMI
        torch.cuda.synchronize()
    return kmeranno.SignatureTable.wrap_device(slots.data_ptr(), nb, K, dev.index), slots


def timed(step, ws, args, world, stream, dev, before=None, after=None):
    """W warmup steps, then exactly K steps between barrier + synchronize; then the same K steps
    again with the library's per-phase hipEvents. Max over ranks of (wall s, GPU ms, probe ms
    per call, rest ms per call)."""
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if before is not None:
        before()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    if after is not None:
        after()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    ws.timing(True)
    for _ in range(args.steps):
        step()
    n_t, probe_ms, rest_ms = ws.timing_read()
    ws.timing(False)
    stats = torch.tensor([elapsed, gpu_ms, probe_ms / max(n_t, 1), rest_ms / max(n_t, 1)],
                         dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    return stats.tolist()


def bench_contigs(args, rank, world, dev, stream, sp):
    total_bp, n_contig, seed, t_size, n_fid = 5_000_000, 20, 3, 10_000_000, 10_000
    t0 = time.perf_counter()
    wl = synth.make_contig_workload(total_bp, n_contig, seed + 1000 * rank, t_size, n_fid, K)
    n_bases = int(wl.offsets[-1] - wl.offsets[0])
    n_win = kmeranno.contig_window_count(wl.offsets, K)
    n_probe = synth.probed_windows(wl.dna, wl.offsets, K)
    log(f"[rank {rank}] workload c3: {n_bases} bp in {n_contig} contigs, {len(wl.genes)} planted "
        f"genes, {n_win} 6-frame windows ({n_probe} probed), generated in "
        f"{time.perf_counter() - t0:.1f}s")
    table, slots = build_table(wl.keys, wl.fids, t_size, args.load_factor, dev, sp, rank, world)
    ws = kmeranno.Workspace(dev.index)
    ws.reserve_contigs(n_bases)
    d_dna = torch.from_numpy(wl.dna).to(dev)
    d_off = torch.from_numpy(wl.offsets.view(np.int64)).to(dev)
    cap = max(1 << 16, n_probe // 4)
    d_hits = torch.empty(cap * kmeranno.HIT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    d_nh = torch.zeros(1, dtype=torch.int64, device=dev)

    def step():
        kmeranno.annotate_contigs_device(table, ws, d_dna.data_ptr(), d_off.data_ptr(), n_contig,
                                         n_bases, 11, d_hits.data_ptr(), cap, d_nh.data_ptr(),
                                         0, 0, sp)

    elapsed, gpu_ms, k1_ms, rest_ms = timed(step, ws, args, world, stream, dev)
    n_hits = int(d_nh.item())
    assert n_hits <= cap, "hit buffer too small"
    if rank == 0:
        value = n_win * args.steps * world / elapsed
        # Probe kernel algorithmic bytes: one 64-B bucket per probed window, 1 B per base read,
        # one 8-B staged record per hit.
        alg_bytes = n_probe * BYTES_PER_LOOKUP + n_bases + 8 * n_hits
        achieved = alg_bytes / (k1_ms * 1e-3) / 1e9
        kname = f"contigs_probe_quad_kernel<{K}, {table.info.minimizer_len}>"
        traffic = None
        try:
            traffic = json.load(open(TRAFFIC_FILE))["workloads"]["c3"][kname]["traffic_bytes"]
        except (OSError, KeyError, ValueError):
            pass
        out = {
            "metric": "kmer lookups/s + seqs annotated/s at 1/2/4/8 GPUs; achieved HBM GB/s vs "
                      "roofline",
            "value": value, "unit": "kmer lookups/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (seeded; SURVEY.md §8(d) config 3 generator)",
            "config": {"workload": f"c3: {WORKLOADS['c3']}", "bases_per_gpu": n_bases,
                       "contigs_per_gpu": n_contig, "windows_per_gpu": n_win,
                       "probed_windows_per_gpu": n_probe, "hits_per_gpu": n_hits,
                       "table_entries": t_size, "functions": n_fid, "k": K,
                       "genetic_code": 11, "load_factor": args.load_factor,
                       "parallelism": f"genome-shard x{world}, table replicated (RCCL broadcast)"},
            "seqs_per_s": n_contig * args.steps * world / elapsed,
            "gpu_ms_per_step": gpu_ms / args.steps,
            "phases_ms": {"probe": k1_ms, "scan_emit": rest_ms},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": f"{os.path.relpath(TRAFFIC_FILE, ROOT)} (rocprofv3 "
                                           "FETCH_SIZE + WRITE_SIZE per launch, calibrated)",
                         "kernel": f"{kname} (6-frame translate + 2 probes per base)",
                         "kernel_ms": k1_ms, "alg_bytes_per_launch": alg_bytes,
                         "measured_random_64B_ceiling_GBps": GATHER_CEILING_GBS},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_contigs(wl)
        print(json.dumps(out), flush=True)
    ws.close()
    table.close()
    del slots


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--load-factor", type=float, default=0.5)
    ap.add_argument("--n-seq", type=int, default=0,
                    help="override the workload's proteins per rank (tuning runs only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream

    if args.workload == "c3":
        bench_contigs(args, rank, world, dev, stream, sp)
        if world > 1:
            dist.destroy_process_group()
        return

    n_seq, t_size, n_fid, seed = synth.CONFIGS[args.workload]
    n_seq = args.n_seq or n_seq
    t0 = time.perf_counter()
    sig = synth.make_table(t_size, n_fid, seed, K)
    residues, offsets, _, _ = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17 + rank)
    lens = np.diff(offsets).astype(np.int64)
    n_win = int(np.maximum(lens - K + 1, 0).sum())
    log(f"[rank {rank}] workload {args.workload}: {t_size} table rows, {n_seq} proteins, "
        f"{n_win} windows, generated in {time.perf_counter() - t0:.1f}s")
    table, slots = build_table(sig.keys, sig.fids, t_size, args.load_factor, dev, sp, rank, world)
    n_res = int(offsets[-1] - offsets[0])
    ws = kmeranno.Workspace(local, n_res)

    d_res = torch.from_numpy(residues).to(dev)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    d_fid = torch.empty(n_seq, dtype=torch.int32, device=dev)
    d_cnt = torch.empty(n_seq, dtype=torch.int32, device=dev)
    d_st = torch.empty(n_seq, dtype=torch.uint8, device=dev)
    d_tally = torch.zeros(n_fid, dtype=torch.int32, device=dev)

    def step():
        kmeranno.annotate_proteins_device(table, ws, d_res.data_ptr(), d_off.data_ptr(), n_seq,
                                          n_res, MIN_HITS, 0, d_fid.data_ptr(), d_cnt.data_ptr(),
                                          d_st.data_ptr(), d_tally.data_ptr(), n_fid, sp)

    # per-function tallies of the whole job -> rank 0, inside the timed region
    reduce = (lambda: kdist.reduce_tallies(d_tally, dst=0)) if world > 1 else None
    elapsed, gpu_ms, k1_ms, k2_ms = timed(step, ws, args, world, stream, dev,
                                        before=d_tally.zero_, after=reduce)

    fused = ws.protein_form(n_seq) == 1
    st = d_st.cpu().numpy()
    called = int((st == kmeranno.STATUS_CALLED).sum())
    if rank == 0:
        total_lookups = n_win * args.steps * world
        value = total_lookups / elapsed
        seqs_per_s = n_seq * args.steps * world / elapsed
        n_pos = max(n_res - K + 1, 0)
        # K1 algorithmic bytes per launch: one 64-B bucket line + the 4-B result word per residue
        # position probed, + 1 B per residue streamed in.
        alg_bytes = n_pos * (BYTES_PER_LOOKUP + 4) + n_res
        achieved = alg_bytes / (k1_ms * 1e-3) / 1e9
        m = table.info.minimizer_len
        if fused:
            k1_name = f"annotate_kernel<{K}, {m}, 4>"
        else:
            k1_name = os.environ.get("KMA_PROBE", "quad")
            k1_name = {"lane": "probe_kernel", "run": "probe_run_kernel"}.get(
                k1_name, "probe_quad_kernel")
            k1_name = f"{k1_name}<{K}, {m}, 3>"
        traffic = None
        try:
            tr = json.load(open(TRAFFIC_FILE))["workloads"][args.workload][k1_name]
            traffic = tr["traffic_bytes"]
        except (OSError, KeyError, ValueError):
            pass
        out = {
            "metric": "kmer lookups/s + seqs annotated/s at 1/2/4/8 GPUs; achieved HBM GB/s vs "
                      "roofline",
            "value": value,
            "unit": "kmer lookups/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded; SURVEY.md §8(d) generator)",
            "config": {"workload": f"{args.workload}: {WORKLOADS[args.workload]}",
                       "proteins_per_gpu": n_seq, "windows_per_gpu": n_win,
                       "table_entries": t_size, "functions": n_fid, "k": K,
                       "load_factor": args.load_factor, "min_hits": MIN_HITS,
                       "parallelism": f"input-shard x{world}, table replicated (RCCL broadcast), "
                                      "tally reduce (RCCL)"},
            "seqs_per_s": seqs_per_s,
            "called_per_batch": called,
            "gpu_ms_per_step": gpu_ms / args.steps,
            "phases_ms": ({"probe_vote_K12": k1_ms, "vote_long": k2_ms} if fused else
                          {"probe_K1": k1_ms, "vote_K2": k2_ms}),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": f"{os.path.relpath(TRAFFIC_FILE, ROOT)} (rocprofv3 "
                                           "FETCH_SIZE + WRITE_SIZE per launch, calibrated)",
                         "kernel": f"{k1_name} " + ("(K12: every window's bucket gather + the "
                                                    "vote, fused)" if fused else
                                                    "(K1: every window's bucket gather)"),
                         "kernel_ms": k1_ms, "alg_bytes_per_launch": alg_bytes,
                         "measured_random_64B_ceiling_GBps": GATHER_CEILING_GBS},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(sig, residues, offsets)
        print(json.dumps(out), flush=True)
    ws.close()
    table.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
