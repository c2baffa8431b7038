#!/usr/bin/env python3
"""Per-kernel average durations from rocprofv3 --stats CSVs under a directory."""
import csv, glob, os, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
    print(os.path.dirname(f))
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "kma" in n:
            print(f"    {n.replace('kma::(anonymous namespace)::', '')[:44]:44s} {r['Calls']:>4s} "
                  f"{float(r['AverageNs']) / 1e3:10.1f} us")
