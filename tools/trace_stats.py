#!/usr/bin/env python3
"""Per-dispatch statistics of one kernel from a rocprofv3 kernel trace (csv): duration
median/mean/min/max, gaps between consecutive dispatches, medians over windows of dispatches.

Usage: python3 tools/trace_stats.py RUN_kernel_trace.csv [KERNEL_NAME_SUBSTRING] [GRID_SIZE_X] [--json OUT]
GRID_SIZE_X keeps only the dispatches of that grid (work-items): one launch size, e.g. the
headline's 1,048,576-record decode (16,384 two-wave blocks = 2,097,152 work-items).
"""
import csv
import statistics
import sys


def main():
    argv = sys.argv[1:]
    out = None
    if "--json" in argv:
        k = argv.index("--json")
        out = argv[k + 1]
        argv = argv[:k] + argv[k + 2:]
    path = argv[0]
    pat = argv[1] if len(argv) > 1 else "spec_decode_flat"
    grid = int(argv[2]) if len(argv) > 2 else None
    rows = [r for r in csv.DictReader(open(path))
            if pat in r["Kernel_Name"] and (grid is None or int(r["Grid_Size_X"]) == grid)]
    if not rows:
        print("no dispatches match", pat)
        return
    st = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    durs = [(e - s) / 1e3 for s, e in st]
    print(f"{pat}: {len(durs)} dispatches, duration us: median {statistics.median(durs):.1f} "
          f"mean {statistics.mean(durs):.1f} min {min(durs):.1f} max {max(durs):.1f}")
    gaps = [(st[i + 1][0] - st[i][1]) / 1e3 for i in range(len(st) - 1)]
    close = [g for g in gaps if g < 1000]
    if close:
        print(f"gaps (<1 ms) us: median {statistics.median(close):.1f} n {len(close)}")
    if out:
        import json

        json.dump({"kernel": pat, "grid_size_x": grid, "dispatches": len(durs),
                   "median_us": round(statistics.median(durs), 3), "mean_us": round(statistics.mean(durs), 3),
                   "min_us": round(min(durs), 3), "max_us": round(max(durs), 3)}, open(out, "w"), indent=1)
    w = max(1, len(durs) // 12)
    for i in range(0, len(durs), w):
        seg = durs[i:i + w]
        print(f"  [{i:5d}..{i + len(seg):5d}) median {statistics.median(seg):.1f} us")


if __name__ == "__main__":
    main()
