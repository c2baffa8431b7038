#!/usr/bin/env python3
"""Per-case TCC counters of a rocprofv3 --pmc run of scripts/layout_sweep.py.

The sweep launches annotate_kernel `launches` times per case, cases in the order its JSON
lines are printed, so the kernel's dispatches (sorted by id) split into consecutive groups.
Prints one JSON line per case: the sweep record plus fabric read requests (TCC_EA0_RDREQ),
L2 hits / misses per launch, and requests per window.

  python scripts/sweep_pmc_summary.py <pmc dir> <sweep stdout log> > profiles/...jsonl
"""
import collections
import csv
import glob
import json
import sys


def main():
    pmc_dir, log = sys.argv[1], sys.argv[2]
    cases = []
    for line in open(log):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            if "launches" in d:
                cases.append(d)
    files = glob.glob(f"{pmc_dir}/**/*counter_collection.csv", recursive=True)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in files:
        for r in csv.DictReader(open(f)):
            if "annotate_kernel" not in r["Kernel_Name"]:
                continue
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(per)
    i = 0
    for c in cases:
        n = c["launches"]
        grp = ids[i:i + n]
        i += n
        if len(grp) < n:
            break
        mean = {k: sum(per[d][k] for d in grp) / n for k in per[grp[0]]}
        req = mean.get("TCC_EA0_RDREQ_sum")
        out = dict(c)
        out.update({"pmc_launches": n, "fabric_requests": req,
                    "l2_hits": mean.get("TCC_HIT_sum"), "l2_misses": mean.get("TCC_MISS_sum"),
                    "requests_per_window": req / c["windows"] if req else None})
        print(json.dumps(out))


if __name__ == "__main__":
    main()
