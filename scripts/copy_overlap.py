#!/usr/bin/env python3
"""Timeline of host calls from a rocprofv3 --kernel-trace --memory-copy-trace run (CSV): calls
are split at gaps > 1 ms; for each call, the H2D copies (count, bytes, busy time, rate while
busy), the kernels (count, busy time), their overlap, the D2H, and the span from the first
copy to the last event.   python scripts/copy_overlap.py <rocprofv3 output dir>"""
import csv
import glob
import json
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def col(r, *names):
    for n in names:
        for k in r:
            if k.lower() == n.lower():
                return r[k]
    raise KeyError(names)


def busy(iv):
    """Length of the union of intervals."""
    tot, end = 0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def main():
    root = sys.argv[1]
    ev = []
    for r in rows(root + "/**/*memory_copy_trace.csv"):
        d = col(r, "Direction", "Kind", "Operation")
        ev.append(("d2h" if "DEVICE_TO_HOST" in d.upper() or "D2H" in d.upper() else
                   "h2d" if "HOST_TO_DEVICE" in d.upper() or "H2D" in d.upper() else d,
                   int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp")),
                   int(r.get("Bytes") or r.get("Size") or 0)))
    for r in rows(root + "/**/*kernel_trace.csv"):
        ev.append(("kernel:" + col(r, "Kernel_Name")[:40], int(col(r, "Start_Timestamp")),
                   int(col(r, "End_Timestamp")), 0))
    ev.sort(key=lambda e: e[1])
    calls, cur, last_end = [], [], None
    for e in ev:
        if cur and e[1] - last_end > 1_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
        last_end = e[2] if last_end is None or not cur[:-1] else max(last_end, e[2])
    if cur:
        calls.append(cur)
    for c in calls:
        h2d = [(a, b) for k, a, b, _ in c if k == "h2d"]
        ker = [(a, b) for k, a, b, _ in c if k.startswith("kernel:annotate") or
               k.startswith("kernel:void kma::(anonymous namespace)::annotate")]
        kall = [(a, b) for k, a, b, _ in c if k.startswith("kernel:")]
        if not h2d or not kall:
            continue
        nbytes = sum(n for k, _, _, n in c if k == "h2d")
        hb, kb = busy(h2d), busy(kall)
        both = hb + kb - busy(h2d + kall)
        t0 = min(a for _, a, _, _ in c)
        print(json.dumps({
            "span_ms": (max(b for _, _, b, _ in c) - t0) / 1e6,
            "h2d": {"n": len(h2d), "bytes": nbytes, "busy_ms": hb / 1e6,
                    "GBps_while_busy": nbytes / hb if hb else None,
                    "first_ms": (min(a for a, _ in h2d) - t0) / 1e6,
                    "last_end_ms": (max(b for _, b in h2d) - t0) / 1e6},
            "kernels": {"n": len(kall), "annotate_n": len(ker), "busy_ms": kb / 1e6,
                        "first_start_ms": (min(a for a, _ in kall) - t0) / 1e6,
                        "last_end_ms": (max(b for _, b in kall) - t0) / 1e6},
            "overlap_ms": both / 1e6,
            "d2h": [((a - t0) / 1e6, (b - a) / 1e6, n) for k, a, b, n in c if k == "d2h"][:4],
            "h2d_ms_each": sorted(round((b - a) / 1e6, 4) for a, b in h2d)[::max(1, len(h2d) // 8)],
            "kernel_ms_each": [round((b - a) / 1e6, 4) for a, b in sorted(ker)],
            "timeline": [(k[:22], round((a - t0) / 1e6, 3), round((b - t0) / 1e6, 3))
                         for k, a, b, _ in c if k != "h2d"][:40],
        }))


if __name__ == "__main__":
    main()
