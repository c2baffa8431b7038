"""Test helpers: oracle tables restricted to the kmers a batch can look up.

A signature table of 10^7-10^8 rows is too large for the scalar C oracle's chained String map
(one malloc per row), but a batch's answer only depends on the rows whose kmer occurs as one
of its windows: every other lookup misses either way. `restricted_oracle_table` keeps those
rows, in file order (so duplicate keys still resolve last-wins), and builds the oracle's
HashMap from them. Windows that straddle two proteins are included too (a harmless superset).
"""
from __future__ import annotations

import numpy as np

K = 8


def batch_window_keys(residues: np.ndarray, k: int = K) -> np.ndarray:
    """Packed keys (standard 5-bit codes) of every k-window of the concatenated residues
    (windows with a byte outside A-Z / '*' get code 0 bits and simply never match)."""
    b = residues.astype(np.int64)
    codes = np.where((b >= 65) & (b <= 90), b - 64, np.where(b == 42, 27, 0)).astype(np.uint64)
    n = len(codes) - k + 1
    if n <= 0:
        return np.zeros(0, np.uint64)
    key = np.zeros(n, np.uint64)
    for j in range(k):
        key = (key << np.uint64(5)) | codes[j:j + n]
    return key


def unpack_keys(keys: np.ndarray, k: int = K) -> np.ndarray:
    """(n, k) uint8 ASCII kmers of packed standard keys."""
    out = np.zeros((len(keys), k), np.uint8)
    for j in range(k):
        out[:, j] = ((keys >> np.uint64(5 * (k - 1 - j))) & np.uint64(31)).astype(np.uint8) + 64
    out[out == 64 + 27] = ord("*")
    return out


def restricted_oracle_table(oracle_c, keys: np.ndarray, fids: np.ndarray, residues: np.ndarray,
                            k: int = K):
    """The oracle's HashMap of the table rows (keys[r], fids[r]) whose key is a window of the
    batch, rows in file order."""
    wk = np.unique(batch_window_keys(residues, k))
    keep = np.isin(keys, wk)
    rows = unpack_keys(keys[keep], k)
    n = len(rows)
    return oracle_c.Table.from_buffer(rows.tobytes(), np.arange(n + 1, dtype=np.uint64) * k,
                                      fids[keep].astype(np.int32))


def full_oracle_table(oracle_c, keys: np.ndarray, fids: np.ndarray, k: int = K):
    """The oracle's HashMap of every table row, in file order (10^8 rows load in ~20 s on the
    GPU box's host: cheaper than restricting them to a whole 1M-protein batch's windows)."""
    rows = unpack_keys(keys, k)
    n = len(rows)
    return oracle_c.Table.from_buffer(rows.tobytes(), np.arange(n + 1, dtype=np.uint64) * k,
                                      fids.astype(np.int32))


def take_proteins(residues: np.ndarray, offsets: np.ndarray, idx: np.ndarray):
    """(residues padded by 32 bytes, offsets) of the proteins idx of a batch, in idx order."""
    idx = np.asarray(idx, np.int64)
    lo, hi = offsets[idx].astype(np.int64), offsets[idx + 1].astype(np.int64)
    lens = hi - lo
    off = np.zeros(len(idx) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    src = np.repeat(lo - off[:-1].astype(np.int64), lens) + np.arange(int(lens.sum()))
    return np.concatenate([residues[src], np.zeros(32, np.uint8)]), off
