"""Host simulation of home-bucket orders for the protein probe (round 6).

For a K = 8 table of T random 8-mers over the 20 standard amino acids at load factor 0.5 (c5:
T = 10^8, 25M buckets, a minimizer picks a 128-byte pair of buckets and the key's parity the
bucket), and for random query proteins of small.gto's CDS lengths, reports per order:
  density  : fraction of probed windows whose home LINE (bucket pair) differs from the previous
             window's in the same protein (the minimizer layout's line requests per window)
  overflow : keys beyond 8 per bucket / T (the keys a two-choice build must place in their
             alternate bucket at least; the build's evictions add to it); and beyond 16 per
             bucket pair, were a pair one 128-byte home
Orders (kma_internal.h minimizer_hash and its round-6 alternatives):
  random   : smallest multiplicative hash of the K - m + 1 m-mers (the shipped order, m = 6)
  syncmer  : closed syncmers first (an m-mer whose smallest 3-mer hash sits at its first or last
             position), then by hash (round 5's measured variant)
  mod      : mod-sampling (Groot Koerkamp & Pibiri 2024): x = position of the smallest 3-mer hash
             among the key's K - 2 3-mers, the m-mer at x mod (K - m + 1) is the minimizer
  mod1     : mod-sampling over single residues (t = 1): x = position of the smallest rank
             31 - code among the key's K residues (ties: the first), the m-mer at x mod 3
             (shipped); mod1id / mod1rare: the same with the codes / rarest-first as ranks
  m5       : random order with m = 5 (128-byte homes of a lower density)
Usage: python scripts/order_sim.py [T] [n_proteins] [order,order,...] [skew]
  skew: residues drawn with UniProt's amino-acid frequencies (default: uniform, as synth.py)
"""
import sys

import numpy as np

U32 = np.uint32
M32 = np.uint64(0xFFFFFFFF)


def mul32(a, c):
    return ((a.astype(np.uint64) * np.uint64(c)) & M32).astype(U32)


def mmer_hash(sub):
    return mul32(sub, 0x9E3779B1)


def mix32_lite(h):
    h = h ^ (h >> U32(16))
    h = mul32(h, 0x7FEB352D)
    return h ^ (h >> U32(15))


def sub_at(keys, k, m, p):
    return ((keys >> np.uint64(5 * (k - m - p))) & np.uint64((1 << (5 * m)) - 1)).astype(U32)


def order_value(keys, order, k=8):
    if order in ("random", "m5"):
        m = 6 if order == "random" else 5
        v = np.full(len(keys), 0xFFFFFFFF, U32)
        for p in range(k - m + 1):
            v = np.minimum(v, mmer_hash(sub_at(keys, k, m, p)))
        return v
    m, s = 6, 3
    g = [mmer_hash(sub_at(keys, k, s, i)) for i in range(k - s + 1)]  # 3-mer hashes
    if order == "syncmer":
        v = np.full(len(keys), 0xFFFFFFFF, U32)
        for p in range(k - m + 1):
            ends = np.minimum(g[p], g[p + m - s])
            mids = np.minimum.reduce([g[p + i] for i in range(1, m - s)])
            closed = ends <= mids
            h = mmer_hash(sub_at(keys, k, m, p)) >> U32(1)
            v = np.minimum(v, np.where(closed, h, h | U32(0x80000000)))
        return v
    if order == "mod":  # round 6's first mod-sampling build (t = 3; replaced by mod1)
        w = k - m + 1
        best = np.full(len(keys), 0xFFFFFFFF, U32)
        for i in range(k - s + 1):
            t3 = sub_at(keys, k, s, i)
            best = np.minimum(best, (mul32(t3, 0x9E3779) & U32(0xFFFFFFF8)) | U32(i))
        p = ((best & U32(7)) % U32(w)).astype(np.uint64)
        return mmer_hash(((keys >> (np.uint64(5) * (np.uint64(k - m) - p)))
                          & np.uint64((1 << (5 * m)) - 1)).astype(U32))
    if order in ("mod1", "mod1id", "mod1rare"):  # kma_internal.h mod_sample (t = 1): ranks
        # 31 - code; mod1id: the codes themselves; mod1rare: rarest residue (UniProt) first
        rank = {"mod1": lambda c: U32(31) - c, "mod1id": lambda c: c, "mod1rare": lambda c: RARE[c]}
        best = np.full(len(keys), 0xFFFFFFFF, U32)
        for i in range(k):
            c = sub_at(keys, k, 1, i)
            best = np.minimum(best, (rank[order](c) << U32(3)) | U32(i))
        p = ((best & U32(7)) % U32(3)).astype(np.uint64)
        return mmer_hash(((keys >> (np.uint64(5) * (np.uint64(k - m) - p)))
                          & np.uint64((1 << (5 * m)) - 1)).astype(U32))
    raise ValueError(order)


def pair_of(v, nb):
    return ((mix32_lite(v ^ U32(0x85EBCA77)).astype(np.uint64) * np.uint64(nb >> 1)) >> np.uint64(32))


def parity(keys):
    x = (keys & M32).astype(np.uint64)
    c = np.zeros(len(keys), np.uint64)
    while True:
        nz = x != 0
        if not nz.any():
            break
        c[nz] ^= np.uint64(1)
        x &= x - np.uint64(1)
    return c


# UniProtKB/Swiss-Prot amino-acid composition (%), A C D E F G H I K L M N P Q R S T V W Y
UNIPROT = np.array([8.25, 1.37, 5.45, 6.75, 3.86, 7.07, 2.27, 5.96, 5.84, 9.66, 2.42, 4.06, 4.70,
                    3.93, 5.53, 6.56, 5.34, 6.87, 1.08, 2.92])
PROBS = None  # None: uniform residues
RARE = np.full(32, 31, U32)  # residue code -> rank by UniProt frequency (rarest 0)
for _r, _i in enumerate(np.argsort(UNIPROT, kind="stable")):
    RARE[b"ACDEFGHIKLMNPQRSTVWY"[_i] - 64] = _r


def residues(rng, n):
    return rng.integers(0, 20, n) if PROBS is None else rng.choice(20, n, p=PROBS)


def random_kmers(rng, n, k=8):
    key = np.zeros(n, np.uint64)
    codes = (np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8).astype(np.uint64) - 64)
    for _ in range(k):
        key = (key << np.uint64(5)) | codes[residues(rng, n)]
    return key


def main():
    global PROBS
    if len(sys.argv) > 4 and sys.argv[4] == "skew":
        PROBS = UNIPROT / UNIPROT.sum()
    T = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    n_prot = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000
    nb = (T + 3) // 4  # 8 slots, load factor 0.5
    nb += nb & 1
    rng = np.random.default_rng(5)
    sys.path.insert(0, "kmers.anno_amd/python")
    from kmeranno import synth
    lens = rng.choice(synth.cds_lengths(), n_prot)
    aa = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    qkeys = [synth.window_keys(aa[residues(rng, int(L))]) for L in lens]
    orders = sys.argv[3].split(",") if len(sys.argv) > 3 else ("random", "syncmer", "mod", "mod1", "m5")
    for order in orders:
        counts = np.zeros(nb, np.int64)
        chunk = 10_000_000
        krng = np.random.default_rng(55)
        for a in range(0, T, chunk):
            keys = random_kmers(krng, min(chunk, T - a))
            b = 2 * pair_of(order_value(keys, order), nb) + parity(keys)
            counts += np.bincount(b.astype(np.int64), minlength=nb)
        over = np.maximum(counts - 8, 0).sum() / T
        pairs = counts[0::2] + counts[1::2]  # one 128-byte home of 16 slots per pair
        over16 = np.maximum(pairs - 16, 0).sum() / T
        changes = windows = 0
        for q in qkeys:
            pr = pair_of(order_value(q, order), nb)
            changes += 1 + int((pr[1:] != pr[:-1]).sum())
            windows += len(pr)
        print(f"{order:8s} {'skew ' if PROBS is not None else ''}density {changes / windows:.4f}  overflow {over:.4f}  "
              f"overflow of 128-byte homes {over16:.4f}  max keys per bucket {counts.max()}",
              flush=True)


if __name__ == "__main__":
    main()
