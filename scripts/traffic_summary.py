#!/usr/bin/env python3
"""Per-launch HBM traffic of the hot-path kernels from scripts/gpu_traffic.sh's counter runs
(rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_*), calibrated on kma_gather_bench: its kernel
reads a known number of random 64-B lines, so FETCH_SIZE / (lines x 64 B) is the correction for
this access width (MI355X_MICROARCH.md: non-streaming widths are uncalibrated).

  python scripts/traffic_summary.py <dir with pmc_*> <gather lines_per_launch> > profiles/...json
"""
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "kmers.anno_amd", "python"))
import kmeranno  # noqa: E402  (source_digest only: no library load)


def load(d):
    files = glob.glob(d + "/*counter_collection.csv")
    if not files:
        return {}
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for r in csv.DictReader(open(files[0])):
        m = re.search(r"(annotate_kernel<[^>]*>|contigs_\w+_kernel(?:<[^>]*>)?|pack_residues_kernel|"
                      r"gather_\w+)",
                      r["Kernel_Name"])
        if not m:
            continue
        per[m.group(1)][r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in per.items()}


root, lines = sys.argv[1], float(sys.argv[2])
g = load(f"{root}/pmc_gather_FETCH_SIZE")
gk = next(iter(g))
corr = lines * 64 / (g[gk]["FETCH_SIZE"] * 1024)
out = {"source_sha16": kmeranno.source_digest(),
       "calibration": {"kernel": gk, "lines_per_launch": lines,
                       "fetch_bytes": g[gk]["FETCH_SIZE"] * 1024, "factor": corr},
       "workloads": {}}
# every workload tag measured: c2 .. c5, and LF-sweep tags such as c5_lf0.75 (gpu_measure.sh WLS)
tags = sorted({os.path.basename(d)[len("pmc_"):-len("_FETCH_SIZE")]
               for d in glob.glob(f"{root}/pmc_*_FETCH_SIZE")} - {"gather"})
for wl in tags:
    f, w, t = (load(f"{root}/pmc_{wl}_{c}") for c in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum"))
    if not f:
        continue
    ks = {}
    for k in f:
        rd = f[k]["FETCH_SIZE"] * 1024 * corr
        wr = w.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        tc = t.get(k, {})
        hit = tc.get("TCC_HIT_sum", 0.0)
        miss = tc.get("TCC_MISS_sum", 0.0)
        ks[k] = {"read_bytes": rd, "write_bytes": wr, "traffic_bytes": rd + wr,
                 "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
                 "read_requests": tc.get("TCC_EA0_RDREQ_sum"),
                 "read_requests_32B": tc.get("TCC_EA0_RDREQ_32B_sum")}
    out["workloads"][wl] = ks
print(json.dumps(out, indent=1))
