"""CPU, world_size 2 over gloo: residue-balanced sharding, the tally reduce and the result
gather give exactly the single-process answer. The per-shard annotate step is the oracle
here (CPU test); on the GPU box bench.py runs the same host logic around libkmeranno.so."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_shard_bounds_balanced_and_complete():
    from kmeranno import dist, synth
    rng = np.random.default_rng(0)
    lens = rng.choice(synth.cds_lengths(), 5000)
    off = np.zeros(len(lens) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    for world in (1, 2, 3, 8):
        b = dist.shard_bounds(off, world)
        assert b[0] == 0 and b[-1] == len(lens) and (np.diff(b) >= 0).all()
        per = [int(off[b[r + 1]] - off[b[r]]) for r in range(world)]
        assert max(per) - min(per) <= 2 * lens.max()
    empty = dist.shard_bounds(np.zeros(1, np.uint64), 4)
    assert list(empty) == [0, 0, 0, 0, 0]


def _worker(rank, world, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "kmers.anno_amd", "python")]
    import torch
    import torch.distributed as tdist
    from kmeranno import dist, synth
    from oracle import c_oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = synth.make_workload(600, 5000, 200, seed=9)
        kmers = [synth.unpack_key(x) for x in wl.keys]
        table = c_oracle.Table(kmers, wl.fids.astype(np.int32))
        res, off, lo = dist.shard(wl.residues, wl.offsets, world, rank)
        fid, cnt, st = c_oracle.apply(table, res, off, 8, 5, 0)
        tally = torch.from_numpy(np.bincount(fid[st == 1], minlength=200).astype(np.int32))
        dist.reduce_tallies(tally, dst=0)
        g_fid = dist.gather_results(fid, wl.n_seq, lo)
        g_st = dist.gather_results(st, wl.n_seq, lo)
        slots = torch.arange(16, dtype=torch.int64) if rank == 0 else torch.zeros(16, dtype=torch.int64)
        dist.broadcast_table(slots, src=0)
        # the bench's other collectives: per-rank times max-reduced, the layout broadcast
        times = torch.tensor([1.0 + rank, 5.0 - rank], dtype=torch.float64)
        dist.all_reduce_max(times)
        lay = torch.tensor([7 if rank == 0 else 0], dtype=torch.int32)
        dist.broadcast(lay, src=0)
        objs = dist.gather_objects(("r", rank))
        assert times.tolist() == [2.0, 5.0] and int(lay.item()) == 7
        assert objs == ([("r", 0), ("r", 1)] if rank == 0 else None)
        if rank == 0:
            efid, ecnt, est = c_oracle.apply(table, wl.residues, wl.offsets, 8, 5, 0)
            ok = ((g_fid == efid).all() and (g_st == est).all()
                  and (tally.numpy() == np.bincount(efid[est == 1], minlength=200)).all()
                  and (slots.numpy() == np.arange(16)).all())
            q.put(bool(ok))
        else:
            q.put((slots.numpy() == np.arange(16)).all())
    finally:
        tdist.destroy_process_group()


def test_two_rank_gloo_matches_single_process(oracle_c):
    mp = pytest.importorskip("torch.multiprocessing")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(results) and all(p.exitcode == 0 for p in procs)
