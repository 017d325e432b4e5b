#!/usr/bin/env python3
"""The dispatches of the last spec_tree_decoder_run pass in a rocprofv3 kernel trace (csv), in
launch order: kernel, grid, duration.  A pass ends with rows_out_kernel.

Usage: python3 tools/tree_trace.py RUN_kernel_trace.csv [PASSES]
"""
import csv
import sys


def short(name):
    name = name.replace("(anonymous namespace)", "anon")
    return name.split("(")[0].split("::")[-1]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "rows_out_kernel" in r["Kernel_Name"]]
    if not ends:
        print("no rows_out_kernel dispatch")
        return
    for k in range(passes):
        e = ends[-1 - k]
        s = ends[-2 - k] + 1 if len(ends) > 1 + k else 0
        total = 0.0
        t0 = int(rows[s]["Start_Timestamp"])
        print(f"pass ending at dispatch {e}:")
        for r in rows[s:e + 1]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            total += d
            grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
            lds = r.get("LDS_Block_Size", r.get("Lds_Size", "?"))
            print(f"  {short(r['Kernel_Name']):28s} grid {grid:>9s} lds {lds:>6s} {d:9.1f} us")
        wall = (int(rows[e]["End_Timestamp"]) - t0) / 1e3
        print(f"  kernels {total:.1f} us, wall {wall:.1f} us")


if __name__ == "__main__":
    main()
