#!/usr/bin/env python3
"""Per-call timeline of host protein calls from a rocprofv3 --kernel-trace --memory-copy-trace
run (CSV; e.g. scripts/e2e_host.py under rocprofv3). Calls are the groups of events separated
by more than 0.5 ms of silence that contain annotate kernels. For each call: span, H2D copies
(count, busy ms, link idle ms between the first and last copy), kernels, the drain after the
last H2D, and (with --events) every event relative to the call start.

  python scripts/host_call_timeline.py <rocprofv3 output dir> [--events]
"""
import csv
import glob
import json
import sys


def main():
    d = sys.argv[1]
    ev = []
    for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            kind = "H2D" if "HOST_TO_DEVICE" in r["Direction"] else "D2H"
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            kind = "annotate" if "annotate_kernel" in n else ("copy_kernel" if "copyBuffer" in n
                                                               else "other")
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    ev.sort()
    calls, cur = [], [ev[0]]
    for e in ev[1:]:
        if e[0] - max(x[1] for x in cur) > 500_000:
            calls.append(cur)
            cur = [e]
        else:
            cur.append(e)
    calls.append(cur)
    for c in calls:
        if not any(e[2] == "annotate" for e in c):
            continue
        t0 = c[0][0]
        end = max(e[1] for e in c)
        h2d = [e for e in c if e[2] == "H2D"]
        ker = [e for e in c if e[2] == "annotate"]
        busy = sum(e[1] - e[0] for e in h2d)
        out = {
            "span_ms": (end - t0) / 1e6,
            "h2d": {"n": len(h2d), "busy_ms": busy / 1e6,
                    "first_start_ms": (h2d[0][0] - t0) / 1e6 if h2d else None,
                    "last_end_ms": (max(e[1] for e in h2d) - t0) / 1e6 if h2d else None},
            "kernels": {"n": len(ker), "busy_ms": sum(e[1] - e[0] for e in ker) / 1e6,
                        "last_end_ms": (max(e[1] for e in ker) - t0) / 1e6},
        }
        if h2d:
            # link idle: time between the first copy's start and the last copy's end with no copy
            idle, t = 0, h2d[0][0]
            for s, e, _ in h2d:
                if s > t:
                    idle += s - t
                t = max(t, e)
            out["h2d"]["link_idle_ms"] = idle / 1e6
            out["drain_after_last_h2d_ms"] = (end - max(e[1] for e in h2d)) / 1e6
        if "--events" in sys.argv:
            out["events"] = [[round((s - t0) / 1e6, 3), round((e - t0) / 1e6, 3), k]
                             for s, e, k in c]
        print(json.dumps(out))


if __name__ == "__main__":
    main()
