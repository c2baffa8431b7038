#!/usr/bin/env python3
"""Print a short summary of gpurun_out/ (steps, pytest tail, bench lines, kernel stats)."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
p = os.path.join(out, "steps.log")
if os.path.exists(p):
    print("".join(l for l in open(p) if "rc=" in l), end="")
p = os.path.join(out, "pytest_gpu.log")
if os.path.exists(p):
    print("pytest:", open(p).read().strip().splitlines()[-1])
for f in sorted(glob.glob(os.path.join(out, "bench*.log"))):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            r = d["roofline"]
            print(f"{os.path.basename(f)}: {d['config']['workload'][:3]} n={d['n_gpus']} "
                  f"{d['value'] / 1e9:.2f} G lookups/s  {d['ms_per_step']:.4f} ms/step  "
                  f"K1 {r['kernel_ms']:.4f} ms  achieved {r['achieved']:.0f} GB/s frac {r['frac']:.3f}"
                  + (f"  cpu {d['cpu_baseline']['value'] / 1e6:.2f} M/s" if "cpu_baseline" in d else ""))
for f in sorted(glob.glob(os.path.join(out, "**", "*kernel_stats.csv"), recursive=True)):
    print(f)
    for row in csv.DictReader(open(f)):
        if "kma::" in row["Name"]:
            name = row["Name"].split("::")[-1][:60]
            print(f"   {name:60s} calls {row['Calls']:>4s} avg {float(row['AverageNs']) / 1e3:10.1f} us")
p = os.path.join(out, "gather_all.log")
if os.path.exists(p):
    print(open(p).read(), end="")
