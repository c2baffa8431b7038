#!/usr/bin/env python3
"""`kma apply-fasta` loop time over c4's 1M-protein FASTA file for several --callers / --batch /
--threads settings (each run twice, file in the page cache). Prints one JSON line per setting.

  python scripts/fasta_sweep.py "callers batch threads" ...   e.g. "2 16777216 16" "1 67108864 16"
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."),
                os.path.join(os.path.dirname(__file__), "..", "kmers.anno_amd", "python")]
from kmeranno import synth  # noqa: E402

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    settings = [tuple(int(x) for x in a.split()) for a in sys.argv[1:]] or [(2, 16 << 20, 16)]
    n_seq, t_size, n_fid, seed = synth.CONFIGS["c4"]
    root = tempfile.mkdtemp(prefix="kma_fasta_sweep_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        sig = synth.make_table(t_size, n_fid, seed, 8)
        res, off, _, true_fid = synth.make_queries(sig, n_seq, seed * 1_000_003 + 17)
        db, roles, faa = (os.path.join(root, x) for x in ("kmerdb.tbl", "roles", "p.faa"))
        synth.write_kmer_db(db, sig.keys, sig.fids)
        synth.write_roles_in_use(roles, n_fid, every=10)
        synth.write_fasta(faa, res, off, [f"fig|83333.1.peg.{i + 1}" for i in range(n_seq)],
                          [synth.role_name(int(t)) if t >= 0 else "hypothetical protein"
                           for t in true_fid])
        kma = os.path.join(ROOT, "kmers.anno_amd", "build", "kma")
        ref = None
        for callers, batch, threads in settings:
            loops = []
            for _ in range(2):
                p = subprocess.run([kma, "apply-fasta", "--callers", str(callers), "--batch",
                                    str(batch), "--threads", str(threads), db, roles, faa],
                                   capture_output=True, text=True, timeout=600)
                assert p.returncode == 0, p.stderr[-2000:]
                st = json.loads([ln for ln in p.stderr.splitlines()
                                 if "apply-fasta-stats" in ln][0].split("stats ", 1)[1])
                loops.append(st)
                ref = ref or p.stdout
                assert p.stdout == ref, "report differs between settings"
            best = min(loops, key=lambda s: s["loop_s"])
            print(json.dumps({"callers": callers, "batch": batch, "threads": threads,
                              "loop_s": [s["loop_s"] for s in loops], "best": best}), flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
