#!/usr/bin/env python3
"""Per-kernel SQ counter means (per dispatch) from gpu_sq.sh's passes, with the wave-cycle split
(ACTIVE_INST_ANY / WAIT_ANY / WAIT_INST_ANY over WAVE_CYCLES, all quad-cycles) and the
instructions per wave.   python scripts/sq_summary.py gpurun_out/<dir>"""
import collections
import csv
import glob
import json
import re
import sys

root = sys.argv[1]
out = {}
for d in sorted(glob.glob(root + "/sq_*_p*")):
    wl = d.rsplit("/", 1)[1].split("_")[1]
    per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(\w+_kernel)(<[^>]*>)?", r["Kernel_Name"])
            name = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]
            per[name][r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    for k, cs in per.items():
        e = out.setdefault(wl, {}).setdefault(k, {})
        for c, v in cs.items():
            e[c] = sum(v.values()) / len(v)
for wl, ks in out.items():
    for k, e in ks.items():
        wc = e.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if c in e:
                    e[c + "_frac"] = e[c] / wc
        w = e.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                      "SQ_INSTS_SMEM"):
                if c in e:
                    e[c + "_per_wave"] = e[c] / w
json.dump(out, sys.stdout, indent=1, sort_keys=True)
print()
