#!/usr/bin/env python3
"""Benchmark of the signature-kmer annotation hot path on MI355X (BASELINE.json metric).

One step = one annotate pass (ProteinKmers extraction + table probe + vote, the loop of
ApplyKmerProcessor.java:122-147) over one rank's batch of synthetic proteins already resident
in HBM, through the C ABI's device entry point (libkmeranno.so: one kernel launch per pass).
The per-function tallies of the APPLY report accumulate on device across steps and are reduced
to rank 0 over RCCL once, inside the timed region (the only exchange step of the path).

Workloads (BASELINE.json configs; the default is c5, the north-star configuration):
  c5  1M proteins per rank vs the 10^8-entry table (1.5 GiB: HBM random access). Weak scaling:
      every rank its own batch, the table built on rank 0 and broadcast (RCCL over xGMI).
  c2  10k proteins vs the 10^7-entry table (153 MiB: Infinity-Cache resident), weak scaling.
  c4  ONE 1M-protein batch cut into residue-balanced shards across the ranks (strong
      scaling), 10^7-entry table replicated.
  c3  6-frame pass (KmerReference.java:157-203) over a rank's 5 Mbp synthetic genome.

Beside the timed steps, rank 0 of a 1-GPU run also reports
  roofline      the dominant kernel's SURVEY §8(d) algorithmic bytes per launch (64 B per
                probed window + its input) over its hipEvent-timed duration against 8 TB/s
                (`achieved`, `frac`); beside it the HBM bytes it really moves (`traffic`,
                `pmc_frac`: rocprofv3 FETCH_SIZE + WRITE_SIZE passes of these kernel sources,
                committed under profiles/, calibrated per the guide) and the fabric line-request
                rate against the random-64-B ceiling measured live on a buffer of the table's
                size (kma_gather_bench);
  e2e           the host entry point kma_annotate_proteins on the same batch from host memory
                (H2D + kernel + D2H through pinned staging): the PCIe-inclusive rate;
  cpu_baseline  the C restatement of the reference loop (oracle/kma_oracle.c) on all the box's
                host cores (and on one core), on a bounded sample of the same batch and the
                same full table.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c5|c2|c3|c4]
  python bench.py --workload genomes|fasta   (the drop-in's command-level regimes: `kma apply`
                  over a GTO directory / `kma apply-fasta` over a protein FASTA file)
  torchrun --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import fnmatch
import json
import os
import re
import subprocess
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
BYTES_PER_LOOKUP = 64  # one 64-byte bucket line per probed window
MALL_BYTES = 256 << 20  # Infinity Cache: a table below it is served on-die (MI355X_MICROARCH.md)
GATHER_BIN = os.path.join(ROOT, "kmers.anno_amd", "build", "kma_gather_bench")
# Per-launch PMC traffic of the dominant kernels of this build (scripts/gpu_traffic.sh +
# scripts/traffic_summary.py).
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r06_traffic.json")
METRIC = "kmer lookups/s + seqs annotated/s at 1/2/4/8 GPUs; achieved HBM GB/s vs roofline"
WORKLOADS = {
    "c2": "10k synthetic proteins (small.gto CDS length distribution) vs 10M-entry protein "
          "8-mer signature table, 1 MI355X per rank",
    "c3": "whole-contig 6-frame DNA->protein kmer annotation: 5 Mbp synthetic genome per rank "
          "(20 contigs, log-uniform 50 kb-1 Mbp, GC 0.5, 0.05% n, genes planted on both strands "
          "over ~50%, code 11) vs 10M-entry protein 8-mer table",
    "c4": "one 1M-protein metagenome batch input-sharded across the GPUs (residue-balanced), "
          "10M-entry table replicated",
    "c5": "1M proteins per rank vs 10^8-entry multi-function signature table "
          "(HBM random access)",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_threads() -> int:
    """Threads the CPU baseline may use: the box's CPU share (OMP_NUM_THREADS is set to it on
    the GPU box; os.cpu_count() shows the whole machine there), else all cores here."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return max(1, min(16, os.cpu_count() or 1))


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def oracle_table(keys, fids):
    from oracle import c_oracle
    c_oracle.build()
    n = len(keys)
    kmers = np.zeros((n, K), np.uint8)
    for j in range(K):
        kmers[:, j] = ((keys >> np.uint64(5 * (K - 1 - j))) & np.uint64(31)).astype(np.uint8) + 64
    t0 = time.perf_counter()
    table = c_oracle.Table.from_buffer(kmers.tobytes(), np.arange(n + 1, dtype=np.uint64) * K,
                                       fids.astype(np.int32))
    return table, time.perf_counter() - t0


def cpu_baseline(keys, fids, residues, offsets, budget_s=8.0):
    """The C oracle (scalar restatement of ApplyKmerProcessor's table load + loop: chained
    String hash map + per-protein kmer set) over the FULL table, timed on all host cores
    (pthreads over proteins) and on one core, each on a bounded leading sample of the batch."""
    from oracle import c_oracle
    table, load_s = oracle_table(keys, fids)
    lens = np.diff(offsets).astype(np.int64)
    n_seq = len(lens)
    threads = host_threads()

    def rate(nt):
        take = min(n_seq, 200 * nt)
        while True:  # grow the sample until one pass takes >= budget / 4
            sub = offsets[:take + 1].copy()
            t0 = time.perf_counter()
            c_oracle.apply_mt(table, residues, sub, K, MIN_HITS, 0, nt)
            dt = time.perf_counter() - t0
            if dt >= budget_s / 4 or take == n_seq:
                break
            take = min(n_seq, take * 2)
        wins = int(np.maximum(lens[:take] - K + 1, 0).sum())
        total, reps = 0.0, 0
        while total < budget_s and reps < 20:
            t0 = time.perf_counter()
            c_oracle.apply_mt(table, residues, sub, K, MIN_HITS, 0, nt)
            total += time.perf_counter() - t0
            reps += 1
        return wins * reps / total, take, wins, reps

    v_all, take, wins, reps = rate(threads)
    v_one, take1, _, _ = rate(1)
    return {"value": v_all, "unit": "kmer lookups/s", "cores": threads, "kind": "port",
            "single_core_value": v_one,
            "host": {"cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
                     "threads_used": threads},
            "sample": f"oracle/kma_oracle.c orc_apply_mt ({threads} pthreads over proteins) on "
                      f"the first {take} proteins of the rank-0 batch ({wins} windows) x {reps} "
                      f"reps, 1-core figure on the first {take1}; against the same "
                      f"{len(keys)}-row table (String-keyed chained map, load {load_s:.1f}s, "
                      f"untimed)"}


def cpu_baseline_contigs(wl, budget_s=8.0):
    """The C oracle's 6-frame pass (translate + processKmers window filter + String-keyed map
    probe per window, KmerReference.java:157-203) on one host core, over leading contigs."""
    from oracle import c_oracle
    table, load_s = oracle_table(wl.keys, wl.fids)
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
            "host": {"cpu_model": cpu_model(), "os_cpu_count": os.cpu_count()},
            "sample": f"oracle/kma_oracle.c orc_annotate_contigs on leading contigs of the rank-0 "
                      f"genome (1..{take} contigs per rep, {reps} reps, {wins} 6-frame windows) "
                      f"against the same {len(wl.keys)}-row table (load {load_s:.1f}s, "
                      f"untimed)"}


def gather_ceiling(table_bytes: int):
    """Random 64-byte line requests per second the chip serves from a buffer of the table's
    size (kma_gather_bench, quad shape = the probe's; best of 2/4/8 lines in flight), measured
    now, on this GPU: the request-rate ceiling of the probe. None if the binary is missing."""
    if not os.path.exists(GATHER_BIN):
        return None
    mib = max(1, table_bytes >> 20)
    best = None
    for inflight in (2, 4, 8):
        try:
            r = subprocess.run([GATHER_BIN, str(mib), "quad", str(inflight)], capture_output=True,
                               text=True, timeout=120, check=True)
            d = json.loads(r.stdout.strip().splitlines()[-1])
        except (subprocess.SubprocessError, ValueError, IndexError, OSError):
            continue
        if best is None or d["lines_per_s"] > best["lines_per_s"]:
            best = d
    return best


def pmc_traffic(workload: str, kernel: str):
    """(traffic bytes per launch, fabric line requests per launch, source, stale) from the
    committed PMC summary, or Nones. stale: the summary was measured on other kernel sources
    than this tree's (its source_sha16 differs): its numbers are then not reported. workload:
    c2 .. c5, or an LF-sweep tag (c5_lf0.75: c5 at load factor 0.75)."""
    try:
        d = json.load(open(TRAFFIC_FILE))
        recs = d["workloads"][workload]
        names = [n for n in recs if fnmatch.fnmatchcase(n, kernel)]  # kernel: may hold a '*'
        rec = recs[names[0]] if len(names) == 1 else recs[kernel]
    except (OSError, KeyError, ValueError):
        return None, None, None, False
    src = os.path.relpath(TRAFFIC_FILE, ROOT)
    if d.get("source_sha16") != kmeranno.source_digest():
        return None, None, src, True
    return rec["traffic_bytes"], rec.get("read_requests"), src, False


def build_table(keys_np, fids_np, t_size, load_factor, dev, sp, rank, world):
    """Signature table built on rank 0's GPU with the library creators' layout rule
    (kmeranno.choose_layout), replicated over RCCL (xGMI) to the other ranks."""
    nb = kmeranno.buckets_for(t_size, load_factor)
    slots = torch.empty(nb * kmeranno.bucket_slots(), dtype=torch.int64, device=dev)
    layout = torch.zeros(1, dtype=torch.int32, device=dev)
    if rank == 0:
        winner = torch.empty(nb * kmeranno.bucket_slots(), dtype=torch.int32, device=dev)
        status = torch.zeros(4, dtype=torch.int32, device=dev)
        keys = torch.from_numpy(keys_np.view(np.int64)).to(dev)
        fids = torch.from_numpy(fids_np.view(np.int32)).to(dev)

        times = {}

        def build(m):
            tb, te = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            tb.record()
            kmeranno.build_device(slots.data_ptr(), nb, winner.data_ptr(), keys.data_ptr(),
                                  fids.data_ptr(), len(keys_np), status.data_ptr(), sp, k=K,
                                  layout=m)
            te.record()
            torch.cuda.synchronize()
            st = status.cpu().numpy().astype(np.int64)
            assert st[0] == 0 or m & kmeranno.LAYOUT_TWO_CHOICE, "table full"
            times[m] = tb.elapsed_time(te)
            return st

        # the library creators' rule (two-choice placement, else size rule then m = 7 / flat
        # rebuilds by measurement)
        m, st = kmeranno.choose_layout(K, nb, build)
        assert st[0] == 0, "table full"
        ms = times[m]
        layout.fill_(m)
        log(f"[rank 0] table: {st[1]} entries, {nb} buckets ({nb * 8 * kmeranno.bucket_slots() / 2**20:.0f} MiB), "
            f"layout m={m & 0xFF}{' two-choice' if m & kmeranno.LAYOUT_TWO_CHOICE else ''}, "
            f"longest chain {st[2]}, displaced {st[3] / max(st[1], 1):.2%}, built in {ms:.1f} ms")
        del winner, keys, fids
    bcast_ms = None
    if world > 1:
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        kdist.broadcast_table(slots, src=0)  # RCCL over xGMI (host-staged under gloo)
        kdist.broadcast(layout, src=0)
        torch.cuda.synchronize()
        bcast_ms = (time.perf_counter() - t0) * 1e3
    m = int(layout.item())
    table = kmeranno.SignatureTable.wrap_device(slots.data_ptr(), nb, K, dev.index, m)
    # the replica's broadcast (this rank's wall time from a common barrier to its copy landing)
    table.broadcast_ms = bcast_ms
    return table, slots


def timed(step, ws, args, world, stream, dev, before=None, after=None):
    """W warmup steps, then exactly K steps between barrier + synchronize; then the same K steps
    again with the library's hipEvents around its kernels. Max over ranks of (wall s, GPU ms,
    main-kernel ms per call, rest ms per call)."""
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
    n_t, phases = ws.phases_read()
    ws.timing(False)
    names = list(phases)
    mine = [elapsed, gpu_ms] + [phases[k] / max(n_t, 1) for k in names]
    stats = torch.tensor(mine, dtype=torch.float64, device=dev)
    if world > 1:
        kdist.all_reduce_max(stats)
    v = stats.tolist()
    timed.ranks = rank_report(mine, args, world, dev)
    return v[0], v[1], dict(zip(names, v[2:]))


def rank_report(mine, args, world, dev):
    """The ranks that joined the timed region (rank, local rank, host, device and its PCI bus),
    each with its own ms per step and main-kernel ms, gathered on rank 0 (None elsewhere and on
    one rank): a scaling record explains itself — which GPUs ran and which one was slowest."""
    if world == 1:
        return None
    import socket
    try:
        props = torch.cuda.get_device_properties(dev)
        name, bus = props.name, getattr(props, "pci_bus_id", None)
    except Exception:  # noqa: BLE001 - identity is best effort
        name, bus = None, None
    me = {"rank": int(os.environ.get("RANK", "0")),
          "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "host": socket.gethostname(),
          "device_index": dev.index, "device": name, "pci_bus_id": bus,
          "ms_per_step": mine[0] * 1e3 / args.steps,
          "kernel_ms": mine[2] if len(mine) > 2 else None}
    return kdist.gather_objects(me)


def roofline(kind, workload, kernel, kernel_ms, alg_bytes, table_bytes, windows, live=True):
    """The dominant kernel's line, by the SURVEY §8(d) rule: achieved = its algorithmic bytes
    per launch (one 64-B bucket line per probed window + the input it streams) / its
    hipEvent-timed mean duration, against the 8 TB/s HBM peak (frac). Minimizer buckets let
    consecutive windows share a line, so the algorithmic figure exceeds the bytes moved.
    traffic = the HBM bytes the kernel really moves per launch (rocprofv3 FETCH_SIZE +
    WRITE_SIZE passes of these kernel sources, committed under profiles/), with pmc_frac =
    traffic / time / peak beside it; the request view: fabric line requests per launch (PMC)
    per second against the random-64-B ceiling measured live on a buffer of the table's size."""
    name = kernel.split(" (")[0]
    traffic, reqs, src, stale = pmc_traffic(workload, re.sub(r"<(\d+), (\d+), \d+, ", r"<\1, \2, *, ", name))
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    ceil = gather_ceiling(table_bytes) if live else None
    out = {"bound": "hbm" if table_bytes > MALL_BYTES else "infinity-cache",
           "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
           "achieved_basis": f"algorithmic bytes per launch ({kind}) / hipEvent kernel time",
           "traffic_source": (f"{src}: rocprofv3 FETCH_SIZE + WRITE_SIZE passes of this kernel "
                              "(MI355X_MICROARCH.md HBM section; Infinity-Cache hits included)")
           if src and not stale else (f"{src} describes other kernel sources: not used"
                                      if stale else None),
           "kernel": kernel, "kernel_ms": kernel_ms, "alg_bytes_per_launch": alg_bytes,
           "windows_per_launch": windows, "table_bytes": table_bytes}
    if traffic:
        out["pmc_GBps"] = traffic / (kernel_ms * 1e-3) / 1e9
        out["pmc_frac"] = out["pmc_GBps"] / HBM_PEAK_GBS
    if reqs:
        out["line_requests_per_launch"] = reqs
        out["line_requests_per_window"] = reqs / windows
    if ceil:
        out["measured_random_64B_ceiling"] = {"lines_per_s": ceil["lines_per_s"],
                                              "GBps": ceil["GBps"], "buffer_MiB":
                                              ceil["buffer_MiB"], "inflight": ceil["inflight"]}
        out["alg_windows_per_s_vs_ceiling"] = windows / (kernel_ms * 1e-3) / ceil["lines_per_s"]
        if reqs:
            rate = reqs / (kernel_ms * 1e-3)
            out["line_requests_per_s"] = rate
            out["requests_frac_of_ceiling"] = rate / ceil["lines_per_s"]
            # the kernel's real bound: fabric line requests against the live
            # random-line ceiling; `frac` keeps SURVEY §8(d)'s algorithmic rule, which exceeds 1
            # for minimizer layouts (windows sharing a home share its line)
            out["frac_requests"] = rate / ceil["lines_per_s"]
            out["bound_by"] = "random line requests (frac_requests)"
    return out


def link_rates(residues, n_res, dev):
    """What bounds the host call: the pinned host -> device rate for the packed stream's bytes
    (one copy, 2 MiB copies, 8 MiB copies over two / four streams) and the host packer's rate
    (kma_pack_residues on one thread and on the staging pool), in GB of residues per second."""
    n_bytes = kmeranno.packed_bytes(n_res)
    src = torch.empty(n_bytes, dtype=torch.uint8).pin_memory()
    dst = torch.empty(n_bytes, dtype=torch.uint8, device=dev)
    src.fill_(1)
    out = {"packed_bytes": n_bytes}
    for name, chunk in (("h2d_one_copy_GBps", n_bytes), ("h2d_2MiB_copies_GBps", 2 << 20)):
        best = None
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for o in range(0, n_bytes, chunk):
                dst[o:o + chunk].copy_(src[o:o + chunk], non_blocking=True)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b)
            best = ms if best is None else min(best, ms)
        out[name] = n_bytes / (best * 1e-3) / 1e9
    n = min(n_res, 64 << 20)
    buf = np.empty(kmeranno.packed_bytes(n), np.uint8)
    buf[:] = 0
    lib = kmeranno.load()
    for key, threads in (("pack_1thread_GBps", 1), ("pack_pool_GBps", 0)):
        with kmeranno.options(host_threads=threads):  # 0: the staging pool's default width
            t0 = time.perf_counter()
            lib.kma_pack_residues(None, residues, n, buf, len(buf))
            out[key] = n / (time.perf_counter() - t0) / 1e9
    # 8 MiB copies alternating over two / four streams (several DMA engines at once?)
    for n_streams in (2, 4):
        streams = [torch.cuda.Stream(dev) for _ in range(n_streams)]
        best = None
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i, o in enumerate(range(0, n_bytes, 8 << 20)):
                with torch.cuda.stream(streams[i % n_streams]):
                    dst[o:o + (8 << 20)].copy_(src[o:o + (8 << 20)], non_blocking=True)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            best = ms if best is None else min(best, ms)
        out[f"h2d_{n_streams}_streams_GBps"] = n_bytes / (best * 1e-3) / 1e9
    out["h2d_bound_ms"] = n_bytes / (max(v for k, v in out.items() if k.startswith("h2d_")) * 1e9) * 1e3
    return out


def kernel_capacity(k, workload):
    """The protein kernel's template capacity P (proteins per block it holds): K = 8 kernels come
    in P = 4 / 6 / 8, the smallest holding the call's block proteins (kma_kernels.hip
    AnnotateLaunch; the library picks 6 per block at c5's size, 4 at c2 / c4's), other K in 8.
    Shown in the kernel name; the PMC summary's record is matched on any P."""
    if k != 8:
        return 8
    return 6 if workload.split("_lf")[0] == "c5" else 4 if workload in ("c2", "c4") else "*"


def protein_roofline(ph, workload, m, n_win, n_res, table_bytes, live=True):
    """Roofline of the protein path's probe kernel (rank 0's shard, times max over ranks)."""
    packed = "pack_kernel" in ph
    return roofline("windows x 64 B + residues (" + ("packed: 0.625 B" if packed else "1 B") +
                    " each)", workload,
                    f"annotate_kernel<{K}, {m}, {kernel_capacity(K, workload)}, "
                    f"{'true' if packed else 'false'}> (probe + sets + vote)",
                    ph["annotate_kernel"], n_win * BYTES_PER_LOOKUP +
                    (n_res * 5 + 7) // 8 if packed else n_win * BYTES_PER_LOOKUP + n_res,
                    table_bytes, n_win, live=live)


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

    elapsed, gpu_ms, ph = timed(step, ws, args, world, stream, dev)
    # one kernel since round 4 (hits emitted by the probe); older libraries: + the emit pass
    k_ms, rest_ms = ph["contigs_probe_kernel"], ph.get("scan_emit", 0.0)
    n_hits = int(d_nh.item())
    assert n_hits <= cap, "hit buffer too small"
    if rank == 0:
        value = n_win * args.steps * world / elapsed
        m = table.info.minimizer_len | (kmeranno.LAYOUT_MOD_SAMPLING
                                        if table.info.minimizer_order else 0)
        kname = f"contigs_probe_quad_kernel<{K}, {m}>"  # M: the order bit rides in m
        out = {
            "metric": METRIC, "value": value, "unit": "kmer lookups/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (seeded; SURVEY.md §8(d) config 3 generator)",
            "config": {"workload": f"c3: {WORKLOADS['c3']}", "bases_per_gpu": n_bases,
                       "contigs_per_gpu": n_contig, "windows_per_gpu": n_win,
                       "probed_windows_per_gpu": n_probe, "hits_per_gpu": n_hits,
                       "table_entries": t_size, "functions": n_fid, "k": K,
                       "genetic_code": 11, "load_factor": args.load_factor,
                       "parallelism": f"genome-shard x{world}" + collective_note(args, world)},
            "seqs_per_s": n_contig * args.steps * world / elapsed,
            "gpu_ms_per_step": gpu_ms / args.steps,
            "phases_ms": {"probe": k_ms, **({"scan_emit": rest_ms} if "scan_emit" in ph else {})},
            # 6-frame probe: one 64-B bucket per probed window, 1 B per base, 16 B per hit
            "roofline": roofline("probed windows x 64 B + bases + hits x 16 B", "c3",
                                 f"{kname} (6-frame translate + 2 probes per base)", k_ms,
                                 n_probe * BYTES_PER_LOOKUP + n_bases + 16 * n_hits,
                                 table.info.bytes, n_probe),
        }
        if world > 1:
            add_rank_fields(out, table, args)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_contigs(wl)
        print(json.dumps(out), flush=True)
    ws.close()
    table.close()
    del slots


def bench_genomes(args):
    """The drop-in's own regime: `kma apply` (the C++ mirror of ApplyKmerProcessor over the C
    ABI) on a directory of synthetic GTOs, as a SEEDtk pipeline runs it (ApplyKmerProcessor.
    java:116-151: genome by genome, every peg's protein). Timed: the command's genome loop
    (parse + native calls + reports; its apply-stats line) in the command's default mode (GTO
    parse-ahead pool, consecutive genomes batched into 16M-residue calls), with each parse
    worker making its own genome's call (--batch 0), and as round 3 ran it (one thread, one
    call per genome).
    The APPLY report is checked line for line against the oracle's calls."""
    import shutil
    import tempfile
    from oracle import c_oracle
    n_gen, pegs = args.genomes, 4000
    t_size, n_fid, seed = 10_000_000, 10_000, 4  # c4's function model and 10^7-row table
    root = tempfile.mkdtemp(prefix="kma_genomes_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        t0 = time.perf_counter()
        sig = synth.make_table(t_size, n_fid, seed, K)
        db, roles, gdir = (os.path.join(root, x) for x in ("kmerdb.tbl", "roles.in.use", "gtos"))
        synth.write_kmer_db(db, sig.keys, sig.fids)
        synth.write_roles_in_use(roles, n_fid, every=10)
        genomes = []
        for a in range(0, n_gen, 50):  # progress every 50 genomes
            genomes += synth.write_genome_dir(gdir, sig, min(50, n_gen - a), pegs, seed=8,
                                              contig_bp=args.contig_bp, first=a)
            log(f"genomes written: {a + min(50, n_gen - a)} ({time.perf_counter() - t0:.0f}s)")
        genomes.sort(key=lambda g: g[0] + ".gto")
        gbytes = sum(os.path.getsize(os.path.join(gdir, f)) for f in os.listdir(gdir))
        n_prot = sum(len(g[2]) - 1 for g in genomes)
        n_win = sum(int(np.maximum(np.diff(g[2]).astype(np.int64) - K + 1, 0).sum())
                    for g in genomes)
        log(f"{n_gen} GTOs ({gbytes / 1e9:.2f} GB), {n_prot} proteins, {n_win} windows, "
            f"generated in {time.perf_counter() - t0:.0f}s")
        kma = os.path.join(ROOT, "kmers.anno_amd", "build", "kma")

        def run(extra, tag):
            out_path = os.path.join(root, f"apply_{tag}.txt")
            with open(out_path, "w") as out:
                p = subprocess.run([kma, "apply", *extra, db, roles, gdir], stdout=out,
                                   stderr=subprocess.PIPE, text=True, timeout=1200)
            if p.returncode != 0:
                raise RuntimeError(f"kma apply {tag}: rc {p.returncode}\n{p.stderr[-3000:]}")
            line = [ln for ln in p.stderr.splitlines() if "apply-stats" in ln][-1]
            stats = json.loads(line.split("apply-stats ", 1)[1])
            log(f"kma apply {tag}: {stats}")
            return stats, open(out_path).read().splitlines()

        dflt, report = run([], "default")
        dflt2, report2 = run([], "default2")  # the GTOs are in the page cache for both
        workers, report_w = run(["--batch", "0"], "worker_calls")
        seq, report_seq = run(["--threads", "1", "--batch", "1"], "per_genome")
        best = min((dflt, dflt2), key=lambda s: s["loop_s"])
        # parity: the oracle's calls (restatement of the same loop) -> the APPLY report
        table, load_s = oracle_table(sig.keys, sig.fids)
        col = {synth.role_name(i): j for j, i in enumerate(range(0, n_fid, 10))}
        expect = []
        for gid, res, off in genomes:
            fid, _, st = c_oracle.apply_mt(table, res, off, K, MIN_HITS, 0, host_threads())
            counts = np.zeros(len(col), np.int64)
            called = fid[st == kmeranno.STATUS_CALLED]
            keep = called[called % 10 == 0] // 10
            np.add.at(counts, keep, 1)
            expect.append(gid + "\t" + "\t".join(map(str, counts.tolist())))
        parity = all(r == expect for r in (report, report2, report_w, report_seq))
        loop = best["loop_s"]
        out = {
            "metric": "genomes annotated/s through `kma apply` (ApplyKmerProcessor mirror over "
                      "the C ABI), GTO directory",
            "value": n_gen / loop, "unit": "genomes/s", "n_gpus": 1, "higher_is_better": True,
            "dtype": "u64", "data": "synthetic GTOs (seeded; SURVEY.md §8(d) protein mix)",
            "config": {"workload": f"genomes: {n_gen} GTOs x {pegs} pegs (small.gto-like, one "
                                   f"{args.contig_bp}-bp contig each) vs the 10^7-row table "
                                   "(c4's function model), roles.in.use of 1,000 roles",
                       "gto_bytes": gbytes, "proteins": n_prot, "windows": n_win,
                       "table_entries": t_size, "k": K, "min_hits": MIN_HITS},
            "seqs_per_s": n_prot / loop, "lookups_per_s": n_win / loop,
            "default_batched": best, "default_runs_loop_s": [dflt["loop_s"], dflt2["loop_s"]],
            "calls_on_parse_workers": dict(workers, genomes_per_s=n_gen / workers["loop_s"]),
            "per_genome_sequential": dict(seq, genomes_per_s=n_gen / seq["loop_s"]),
            "speedup_vs_per_genome": seq["loop_s"] / loop,
            "native_call_share": best["native_call_s"] / loop,
            "apply_report_equals_oracle": parity,
            "oracle_table_load_s": load_s,
        }
        print(json.dumps(out), flush=True)
        if not parity:
            sys.exit(1)
    finally:
        shutil.rmtree(root, ignore_errors=True)


def bench_fasta(args):
    """The FASTA form of the drop-in (north_star: "throughput on synthetic
    FASTA of a stated length distribution"): `kma apply-fasta` as a child process over one
    protein FASTA file of c4's 1M proteins (lengths resampled from small.gto's CDS lengths,
    SURVEY §8(d) query mix, 60-residue lines, ">fig|... function" headers) against c4's
    10^7-row table. Timed: the command's loop, file open -> last report row written (parse,
    native calls, VERIFY rows; its apply-fasta-stats line), best of 2 runs with the file in the
    page cache; the table load is reported beside it. The VERIFY report is checked line for
    line against the oracle's calls on the same proteins."""
    import shutil
    import tempfile
    from oracle import c_oracle
    n_seq, t_size, n_fid, seed = synth.CONFIGS["c4"]
    n_seq = args.n_seq or n_seq
    root = tempfile.mkdtemp(prefix="kma_fasta_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        t0 = time.perf_counter()
        sig = synth.make_table(t_size, n_fid, seed, K)
        res, off, _, true_fid = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
        db, roles, faa = (os.path.join(root, x) for x in ("kmerdb.tbl", "roles.in.use",
                                                             "83333.1.faa"))
        synth.write_kmer_db(db, sig.keys, sig.fids)
        synth.write_roles_in_use(roles, n_fid, every=10)
        ids = [f"fig|83333.1.peg.{i + 1}" for i in range(n_seq)]
        com = [synth.role_name(int(t)) if t >= 0 else "hypothetical protein" for t in true_fid]
        fbytes = synth.write_fasta(faa, res, off, ids, com, width=60)
        n_win = int(np.maximum(np.diff(off).astype(np.int64) - K + 1, 0).sum())
        log(f"FASTA: {n_seq} proteins, {int(off[-1])} residues, {fbytes / 1e6:.0f} MB, "
            f"{n_win} windows; table + file written in {time.perf_counter() - t0:.0f}s")
        kma = os.path.join(ROOT, "kmers.anno_amd", "build", "kma")

        def run(fmt, tag):
            out_path = os.path.join(root, f"report_{tag}.txt")
            w0 = time.perf_counter()
            with open(out_path, "w") as out:
                p = subprocess.run([kma, "apply-fasta", "--format", fmt, db, roles, faa],
                                   stdout=out, stderr=subprocess.PIPE, text=True, timeout=1200)
            wall = time.perf_counter() - w0
            if p.returncode != 0:
                raise RuntimeError(f"kma apply-fasta {tag}: rc {p.returncode}\n{p.stderr[-3000:]}")
            line = [ln for ln in p.stderr.splitlines() if "apply-fasta-stats" in ln][-1]
            stats = json.loads(line.split("apply-fasta-stats ", 1)[1])
            stats["command_wall_s"] = wall
            log(f"kma apply-fasta {tag}: {stats}")
            return stats, open(out_path).read().splitlines()

        runs = [run("VERIFY", f"verify{i}") for i in range(2)]
        apply_stats, apply_report = run("APPLY", "apply")
        best = min(runs, key=lambda r: r[0]["loop_s"])[0]
        table, load_s = oracle_table(sig.keys, sig.fids)
        fid, cnt, st = c_oracle.apply_mt(table, res, off, K, MIN_HITS, 0, host_threads())
        called = np.flatnonzero(st == kmeranno.STATUS_CALLED)
        expect = ["genome_id\tpeg_id\trole\thits\tfunction"] + [
            f"83333.1\t{ids[i]}\t{synth.role_name(int(fid[i]))}\t{int(cnt[i])}\t{com[i]}"
            for i in called]
        counts = np.zeros(len(range(0, n_fid, 10)), np.int64)
        keep = fid[called][fid[called] % 10 == 0] // 10
        np.add.at(counts, keep, 1)
        expect_apply = ["83333.1\t" + "\t".join(map(str, counts.tolist()))]
        parity = all(r[1] == expect for r in runs) and apply_report == expect_apply
        loop = best["loop_s"]
        out = {
            "metric": METRIC, "value": n_win / loop, "unit": "kmer lookups/s", "n_gpus": 1,
            "steps": 1, "warmup": 1, "ms_per_step": loop * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic protein FASTA (seeded; SURVEY.md §8(d) generator: small.gto CDS "
                    "length distribution, 50% mutated prototypes / 40% random / 10% chimeras)",
            "config": {"workload": "fasta: `kma apply-fasta` (file -> VERIFY report) over one "
                                   "FASTA file of c4's 1M proteins vs the 10^7-row table",
                       "proteins": n_seq, "residues": int(off[-1]), "fasta_bytes": fbytes,
                       "windows": n_win, "table_entries": t_size, "k": K, "min_hits": MIN_HITS,
                       "line_width": 60, "parallelism": "one GPU; 4 MiB segments parsed on 16 "
                                                        "host threads, 2 native calls in flight"},
            "seqs_per_s": n_seq / loop, "fasta_mb_per_s": fbytes / 1e6 / loop,
            "loop": best, "runs_loop_s": [r[0]["loop_s"] for r in runs],
            "apply_format": apply_stats,
            "table_load_s": best["table_load_s"],
            "command_wall_s": best["command_wall_s"],
            "native_call_share": best["native_call_s"] / max(loop, 1e-9),
            "verify_report_equals_oracle": all(r[1] == expect for r in runs),
            "apply_report_equals_oracle": apply_report == expect_apply,
            "called": len(called), "oracle_table_load_s": load_s,
        }
        print(json.dumps(out), flush=True)
        if not parity:
            sys.exit(1)
    finally:
        shutil.rmtree(root, ignore_errors=True)


def e2e_host(table, residues, offsets, n_fid, reps=5):
    """kma_annotate_proteins from host memory (H2D + kernel + D2H through the table's pooled
    pinned staging) into the caller's output arrays, reused across calls as a JNI caller reuses
    its direct buffers: best of `reps` calls after one warmup call, in ms, with the library's
    host-side phase profile of that call."""
    n = len(offsets) - 1
    out = (np.empty(n, np.int32), np.empty(n, np.int32), np.empty(n, np.uint8),
           np.zeros(n_fid, np.uint32))
    kmeranno.annotate_proteins(table, residues, offsets, MIN_HITS, 0, n_fid=n_fid, out=out)
    best, prof = 1e30, None
    for _ in range(reps):
        t0 = time.perf_counter()
        kmeranno.annotate_proteins(table, residues, offsets, MIN_HITS, 0, n_fid=n_fid, out=out)
        dt = time.perf_counter() - t0
        if dt < best:
            best = dt
            prof = kmeranno.host_profile()
    e2e_host.profile = prof
    return best * 1e3


def slots_digest(slots) -> int:
    """Order-sensitive checksum of a replica's slot array (sum of slot XOR its index mix)."""
    v = slots.view(torch.int64)
    total, chunk = 0, 1 << 26
    for a in range(0, v.numel(), chunk):
        x = v[a:a + chunk]
        idx = torch.arange(a, a + x.numel(), dtype=torch.int64, device=x.device)
        total = (total + int(torch.bitwise_xor(x, idx * 0x1E3779B97F4A7C15 % (1 << 62)).sum())) % (1 << 64)
    return total


def verify_proteins(args, sig, table, slots, rank, world, strong, full, own, lo, outs, tally_job,
                    n_fid, qseed0):
    """Multi-rank parity of the timed path (--verify), checked on rank 0:
      table    every rank's replica of the broadcast table has the same slot digest and answers
               one probe batch identically (host entry point on each rank);
      outputs  the per-rank outputs (disjoint shards of one batch for c4, each rank's own batch
               for c5 / c2) gathered on rank 0 equal ONE single-rank whole-batch call there;
      tally    the tally reduced over ranks inside the timed region equals steps x the sum of
               the single-rank tallies;
      fan-out  the same whole batch through the host entry point after kma_table_replicate
               added two more replicas on rank 0's device (the ABI's own residue-balanced
               fan-out over replicas, one host thread each) equals the single-replica answer."""
    d_fid, d_cnt, d_st = outs
    mine = (lo, d_fid.cpu().numpy(), d_cnt.cpu().numpy(), d_st.cpu().numpy())
    probe_res, probe_off, _, _ = synth.make_queries(sig, 3000, 4242)
    probe = kmeranno.annotate_proteins(table, probe_res, probe_off, MIN_HITS, 0)[:3]
    digest = slots_digest(slots)
    parts = kdist.gather_objects((mine, probe, digest))
    if rank != 0:
        return None
    out = {"ranks": world}
    out["table_identical_across_ranks"] = bool(
        all(d == parts[0][2] for _, _, d in parts) and
        all(all((a == b).all() for a, b in zip(p, parts[0][1])) for _, p, _ in parts))
    # single-rank answers of the same work
    if strong:
        batches = [full]
    else:  # rank r's own batch is regenerated here from its seed
        batches = [own if r == 0 else synth.make_queries(sig, args.n_seq or len(own[1]) - 1,
                                                         qseed0 + r)[:2]
                   for r in range(world)]
    single, tally = [], np.zeros(n_fid, np.int64)
    for res, off in batches:
        f, c, s, t = kmeranno.annotate_proteins(table, res, off, MIN_HITS, 0, n_fid=n_fid)
        single.append((f, c, s))
        tally += t
    if strong:
        got = [np.concatenate([p[0][i] for p in sorted(parts, key=lambda p: p[0][0])])
               for i in (1, 2, 3)]
        out["outputs_equal_single_rank"] = bool(all((g == e).all()
                                                    for g, e in zip(got, single[0])))
    else:
        out["outputs_equal_single_rank"] = bool(all(
            all((g == e).all() for g, e in zip(parts[r][0][1:], single[r]))
            for r in range(world)))
    out["tally_equals_single_rank"] = bool((tally_job.astype(np.int64) ==
                                            tally * args.steps).all())
    out["called"] = int(sum(int((s[2] == kmeranno.STATUS_CALLED).sum()) for s in single))
    dev = table.info.device
    table.replicate([dev, dev])
    out["replicas"] = table.replicas
    res, off = batches[0]
    fan = kmeranno.annotate_proteins(table, res, off, MIN_HITS, 0, n_fid=n_fid)
    out["replica_fanout_equals"] = bool(all((a == b).all() for a, b in zip(fan[:3], single[0])))
    out["ok"] = all(v for k, v in out.items() if k.endswith(("_ranks", "_rank", "_equals")))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c5",
                    choices=sorted(WORKLOADS) + ["genomes", "fasta"])
    ap.add_argument("--genomes", type=int, default=500,
                    help="genomes workload: GTO files (4,000 pegs each)")
    ap.add_argument("--contig-bp", type=int, default=4_000_000,
                    help="genomes workload: bases of each GTO's contig")
    ap.add_argument("--load-factor", type=float, default=0.5)
    ap.add_argument("--n-seq", type=int, default=0,
                    help="override the workload's proteins per rank (tuning runs only)")
    ap.add_argument("--table-rows", type=int, default=0,
                    help="override the workload's table rows (tests and tuning runs only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the gather ceiling and the host-path (e2e) measurement")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="collectives: nccl = RCCL over xGMI (one GPU per rank); gloo = host-"
                         "staged, to rehearse several ranks on one GPU (with --same-device)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank uses device 0 (multi-rank rehearsal on a 1-GPU box)")
    ap.add_argument("--packed-input", type=int, default=1, choices=(0, 1, 2),
                    help="KMA_OPT_PACKED_INPUT: 1 (default) = batches of >= 2^25 residues are "
                         "packed to 5 bits by a pack kernel inside the step, then the packed "
                         "probe; 2 = every batch; 0 = the probe packs ASCII itself")
    ap.add_argument("--placement", default="auto", choices=("auto", "chained"),
                    help="KMA_OPT_PLACEMENT: auto (default) = two-choice placement for K <= 8 "
                         "tables, chains if that build fails; chained = overflow chains (A/B runs)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="set a library option through the ABI before the run (tuning runs "
                         "only; names as kmeranno._OPT_NAMES, e.g. block_proteins=6)")
    ap.add_argument("--verify", action="store_true",
                    help="after timing, check the multi-rank outputs, tally and table against "
                         "single-rank calls on rank 0 (exit 1 on a mismatch)")
    args = ap.parse_args()

    kmeranno.set_option(kmeranno.OPT_PACKED_INPUT, args.packed_input)
    kmeranno.set_option(kmeranno.OPT_PLACEMENT, 0 if args.placement == "chained" else -1)
    for o in args.option:
        name, _, value = o.partition("=")
        kmeranno.set_option(kmeranno._OPT_NAMES[name], int(value))
    if args.workload == "genomes":  # a command-level run: `kma apply` as a child process
        bench_genomes(args)
        return
    if args.workload == "fasta":  # a command-level run: `kma apply-fasta` as a child process
        bench_fasta(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if args.same_device and world > 1 and args.dist_backend == "nccl":
        ap.error("--same-device needs --dist-backend gloo (RCCL takes one rank per GPU)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream

    if args.workload == "c3":
        bench_contigs(args, rank, world, dev, stream, sp)
        if world > 1:
            dist.destroy_process_group()
        return

    n_seq, t_size, n_fid, seed = synth.CONFIGS[args.workload]
    n_seq = args.n_seq or n_seq
    t_size = args.table_rows or t_size
    strong = args.workload == "c4"
    t0 = time.perf_counter()
    sig = synth.make_table(t_size, n_fid, seed, K, protos_only=rank != 0)
    qseed = seed * 1_000_003 + 17 + (0 if strong else rank)
    residues, offsets, _, _ = synth.make_queries(sig, n_seq, qseed)
    batch_windows = int(np.maximum(np.diff(offsets).astype(np.int64) - K + 1, 0).sum())
    batch_seqs = len(offsets) - 1
    lo = 0
    full = (residues, offsets)  # the whole batch (c4) / this rank's batch (c5, c2)
    if strong:  # this rank's residue-balanced contiguous shard of the one batch
        residues, offsets, lo = kdist.shard(residues, offsets, world, rank)
    n_seq = len(offsets) - 1
    lens = np.diff(offsets).astype(np.int64)
    n_win = int(np.maximum(lens - K + 1, 0).sum())
    log(f"[rank {rank}] workload {args.workload}: {t_size} table rows, {n_seq} proteins "
        f"(from {lo}), {n_win} windows, generated in {time.perf_counter() - t0:.1f}s")
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
    job_tally = torch.zeros_like(d_tally)

    def reduce():
        if world > 1:
            kdist.reduce_tallies(d_tally, dst=0)
        job_tally.copy_(d_tally)

    elapsed, gpu_ms, ph = timed(step, ws, args, world, stream, dev, before=d_tally.zero_,
                                after=reduce)
    st = d_st.cpu().numpy()
    called = int((st == kmeranno.STATUS_CALLED).sum())
    verify = None
    if args.verify:
        verify = verify_proteins(args, sig, table, slots, rank, world, strong, full, full, lo,
                                 (d_fid, d_cnt, d_st), job_tally.cpu().numpy(), n_fid,
                                 seed * 1_000_003 + 17)
    if rank == 0:
        total_lookups = (batch_windows if strong else n_win * world) * args.steps
        value = total_lookups / elapsed
        seqs = batch_seqs if strong else n_seq * world
        # the kernels' minimizer code (length | order bit): their template name in rocprof
        m = table.info.minimizer_len | (kmeranno.LAYOUT_MOD_SAMPLING
                                        if table.info.minimizer_order else 0)
        out = {
            "metric": METRIC, "value": value, "unit": "kmer lookups/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (seeded; SURVEY.md §8(d) generator)",
            "config": {"workload": f"{args.workload}: {WORKLOADS[args.workload]}",
                       "proteins_per_gpu": n_seq, "windows_per_gpu": n_win,
                       "batch_windows": batch_windows if strong else n_win * world,
                       "table_entries": t_size, "functions": n_fid, "k": K,
                       "load_factor": args.load_factor, "min_hits": MIN_HITS,
                       "table_layout_m": table.info.minimizer_len,
                       "table_minimizer_order": "mod-sampling" if table.info.minimizer_order
                       else "random",
                       "table_placement": "two-choice" if table.info.two_choice else "chained",
                       **({"options": args.option} if args.option else {}),
                       "parallelism": (f"input-shard x{world} of one batch" if strong else
                                       f"input-shard x{world}") + collective_note(args, world)},
            "seqs_per_s": seqs * args.steps / elapsed,
            "called_per_batch": called,
            "gpu_ms_per_step": gpu_ms / args.steps,
            "phases_ms": ph,
        }
        wl_tag = args.workload if args.load_factor == 0.5 else f"{args.workload}_lf{args.load_factor:g}"
        out["roofline"] = protein_roofline(ph, wl_tag, m, n_win, n_res, table.info.bytes,
                                           live=not args.no_extras)
        if world > 1:
            add_rank_fields(out, table, args)
        if world == 1:
            if not args.no_extras:
                ms = e2e_host(table, residues, offsets, n_fid)
                prof = e2e_host.profile  # (the ASCII call below replaces it)
                with kmeranno.options(packed_input=0):
                    ms_ascii = e2e_host(table, residues, offsets, n_fid)
                out["e2e_host_call"] = {
                    "entry": "kma_annotate_proteins (host buffers: pinned staging, H2D, kernel, "
                             "D2H, on the table's pooled stream)",
                    "packed_input": kmeranno.get_option(kmeranno.OPT_PACKED_INPUT),
                    "staging_threads": kmeranno.get_option(kmeranno.OPT_HOST_THREADS) or
                    f"min(16, host cores = {kmeranno.host_cores()})",
                    "ms": ms, "library_profile_ms": prof,
                    "lookups_per_s": n_win / (ms * 1e-3),
                    "seqs_per_s": n_seq / (ms * 1e-3), "kernel_ratio": ms / ph["annotate_kernel"],
                    "ascii_staging_ms": ms_ascii,
                    "link": link_rates(residues, n_res, dev)}
            if not args.no_cpu_baseline:
                out["cpu_baseline"] = cpu_baseline(sig.keys, sig.fids, residues, offsets)
        if verify is not None:
            out["verify"] = verify
        print(json.dumps(out), flush=True)
    ws.close()
    table.close()
    if world > 1:
        dist.destroy_process_group()
    if verify is not None and not verify["ok"]:
        sys.exit(1)


def add_rank_fields(out, table, args):
    """Multi-rank lines: the joined ranks (timed.ranks), the spread of their step times and the
    table broadcast's time (rank 0's wall time from a barrier until its copy completed; the
    broadcast sends table.info.bytes to every other rank)."""
    ranks = getattr(timed, "ranks", None) or []
    out["ranks"] = ranks
    steps = [r["ms_per_step"] for r in ranks]
    if steps:
        out["rank_ms_per_step_min"] = min(steps)
        out["rank_ms_per_step_max"] = max(steps)
        out["devices_distinct"] = len({(r["host"], r["pci_bus_id"], r["device_index"])
                                        for r in ranks})
    ms = getattr(table, "broadcast_ms", None)
    out["table_broadcast"] = {"ms": ms, "bytes": table.info.bytes, "backend": args.dist_backend,
                              "GBps_per_receiver": table.info.bytes / (ms * 1e-3) / 1e9
                              if ms else None}


def collective_note(args, world: int) -> str:
    if world == 1:
        return ", table on this GPU"
    if args.dist_backend == "nccl":
        return ", table replicated (RCCL broadcast over xGMI), tally reduce (RCCL)"
    return (", table replicated (gloo broadcast, host-staged), tally reduce (gloo)" +
            ("; every rank on device 0 (multi-rank rehearsal, ranks share one GPU)"
             if args.same_device else ""))


if __name__ == "__main__":
    main()
