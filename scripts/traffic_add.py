"""Add one kernel's traffic entry to profiles/r02_traffic.json from two rocprofv3 --pmc runs:
a TCC pass (TCC_HIT/MISS, TCC_EA0_RDREQ(_32B)) and a WRITE_SIZE pass. Read bytes are the
fabric read requests x 64 B (FETCH_SIZE's definition, MI355X_MICROARCH.md) times the gather
bench calibration already in the file; WRITE_SIZE is in KiB.
  python scripts/traffic_add.py c5 gpurun_out/pmc_m6_req gpurun_out/pmc_m6_wr
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAFFIC = os.path.join(ROOT, "profiles", "r02_traffic.json")


def per_kernel(d):
    """Mean per dispatch of every counter, by kernel (template name as bench.py labels it)."""
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        name = r["Kernel_Name"]
        if "annotate_kernel<" not in name:
            continue
        k = "annotate_kernel<" + name.split("annotate_kernel<")[1].split(">")[0] + ">"
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    wl, req_dir, wr_dir = sys.argv[1:4]
    out = json.load(open(TRAFFIC))
    corr = out["calibration"]["factor"]
    req, wr = per_kernel(req_dir), per_kernel(wr_dir)
    for k, tc in req.items():
        rd = tc["TCC_EA0_RDREQ_sum"] * 64 * corr
        w = wr.get(k, {}).get("WRITE_SIZE", 0.0) * 1024
        hit, miss = tc.get("TCC_HIT_sum", 0.0), tc.get("TCC_MISS_sum", 0.0)
        out["workloads"].setdefault(wl, {})[k] = {
            "read_bytes": rd, "write_bytes": w, "traffic_bytes": rd + w,
            "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
            "read_requests": tc["TCC_EA0_RDREQ_sum"],
            "read_requests_32B": tc.get("TCC_EA0_RDREQ_32B_sum"),
            "source": f"{os.path.basename(req_dir)} + {os.path.basename(wr_dir)}"}
        print(wl, k, out["workloads"][wl][k])
    json.dump(out, open(TRAFFIC, "w"), indent=1)


if __name__ == "__main__":
    main()
