#!/usr/bin/env python3
"""Mean per-dispatch PMC counters per kernel from rocprofv3 --pmc runs.
  python scripts/pmc_summary.py gpurun_out/pmc_c4_*  (dirs with run_counter_collection.csv)"""
import collections
import csv
import glob
import re
import sys

per = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(\w+_kernel)(<[^>]*>)?", r["Kernel_Name"])
            name = m.group(1) if m else r["Kernel_Name"][:40]
            per[name][r["Counter_Name"]][(f, int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
for k, cs in sorted(per.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v.values()) / len(v):16.4g}")
