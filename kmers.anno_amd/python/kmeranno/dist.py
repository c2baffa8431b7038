"""Multi-GPU host logic of the hot path (one process per GPU, torch.distributed over RCCL).

The path shards embarrassingly: proteins are independent, so a batch is cut into contiguous
shards balanced by residue count (not sequence count: lengths are heavy-tailed, 35..2955 aa
in small.gto) and every rank annotates its shard against its own replica of the signature
table. There are exactly two collectives, both outside the per-window data path:
  - the table replica: built once on rank 0, broadcast (ncclBroadcast over xGMI);
  - the APPLY report's per-function tallies: summed to rank 0 (ncclReduce) once per job.
Per-protein outputs need no collective (each rank owns a disjoint slice); gather_results
collects them on rank 0 only when a caller wants one array.
"""
from __future__ import annotations

import numpy as np


def shard_bounds(offsets: np.ndarray, world: int) -> np.ndarray:
    """Protein index bounds [b[r], b[r+1]) of `world` contiguous shards with near-equal
    residue counts (cut where the residue prefix crosses r/world of the total)."""
    offsets = np.asarray(offsets, dtype=np.uint64)
    n = len(offsets) - 1
    total = int(offsets[-1] - offsets[0])
    targets = offsets[0] + (np.arange(1, world, dtype=np.float64) * total / world)
    cuts = np.searchsorted(offsets[1:].astype(np.float64), targets, side="left") + 1
    b = np.concatenate([[0], np.minimum(cuts, n), [n]]).astype(np.int64)
    return np.maximum.accumulate(b)


def shard(residues: np.ndarray, offsets: np.ndarray, world: int, rank: int):
    """(residues slice padded by 32 bytes, rebased offsets, first protein index) of a shard."""
    b = shard_bounds(offsets, world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    r0, r1 = int(offsets[lo]), int(offsets[hi])
    res = np.concatenate([residues[r0:r1], np.zeros(32, np.uint8)])
    off = (offsets[lo:hi + 1] - np.uint64(r0)).astype(np.uint64)
    return res, off, lo


def _multi() -> bool:
    import torch.distributed as dist
    return dist.is_initialized() and dist.get_world_size() > 1


def _staged(collective, tensor, writes_back: bool = True, **kw):
    """Run `collective` on `tensor`. RCCL ("nccl") works on device memory directly; gloo
    (the CPU backend, used to rehearse several ranks on one GPU) has no device reduce, so a
    device tensor is staged through host memory around the collective and copied back where
    the collective defines the result (`writes_back`)."""
    import torch.distributed as dist
    if getattr(tensor, "is_cuda", False) and dist.get_backend() == "gloo":
        host = tensor.cpu()
        collective(host, **kw)
        if writes_back:
            tensor.copy_(host)
    else:
        collective(tensor, **kw)
    return tensor


def broadcast_table(slots, src: int = 0):
    """Replicate the signature table's slot array (a torch tensor) from `src` to every rank
    (RCCL broadcast over xGMI; host-staged under gloo)."""
    import torch.distributed as dist
    if _multi():
        _staged(dist.broadcast, slots, src=src)
    return slots


def broadcast(tensor, src: int = 0):
    """Any small tensor from `src` to every rank (layout choice, flags)."""
    return broadcast_table(tensor, src)


def reduce_tallies(tally, dst: int = 0):
    """Sum the per-function tallies (int32 tensor) of every rank into rank `dst`."""
    import torch.distributed as dist
    if _multi():
        _staged(dist.reduce, tally, writes_back=dist.get_rank() == dst, dst=dst)
    return tally


def all_reduce_max(tensor):
    """Element-wise max over ranks, in place (the bench's per-rank times)."""
    import torch.distributed as dist
    if _multi():
        _staged(dist.all_reduce, tensor, op=dist.ReduceOp.MAX)
    return tensor


def gather_results(local: np.ndarray, n_total: int, lo: int, dst: int = 0):
    """Assemble per-protein arrays (disjoint slices) on rank `dst` (None elsewhere)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return local
    parts = [None] * dist.get_world_size() if dist.get_rank() == dst else None
    dist.gather_object((lo, local), parts, dst=dst)
    if dist.get_rank() != dst:
        return None
    out = np.empty(n_total, dtype=local.dtype)
    for start, arr in parts:
        out[start:start + len(arr)] = arr
    _ = torch  # torch is the transport; numpy holds the result
    return out


def gather_objects(obj, dst: int = 0):
    """Every rank's `obj` as a list on rank `dst` (None elsewhere; [obj] with one rank)."""
    import torch.distributed as dist
    if not _multi():
        return [obj]
    parts = [None] * dist.get_world_size() if dist.get_rank() == dst else None
    dist.gather_object(obj, parts, dst=dst)
    return parts
