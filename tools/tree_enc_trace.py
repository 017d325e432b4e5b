#!/usr/bin/env python3
"""The dispatches of the last spec_encode_tree call in a rocprofv3 kernel trace (csv), in launch
order: kernel, grid, duration, gap before it.  An encode is the size passes, the record scan,
the error check, the position fill and the writers.

Usage: python3 tools/tree_enc_trace.py RUN_kernel_trace.csv
"""
import csv
import sys


def short(name):
    name = name.replace("(anonymous namespace)", "anon")
    return name.split("(")[0].split("::")[-1]


ENC = ("tree_size", "spec_tree_size_set", "scan_tiles", "scan_top", "scan_apply", "tree_err", "tree_pos_fill", "tree_write", "copyBuffer",
       "fillBuffer")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    writes = [i for i, r in enumerate(rows) if "tree_write" in r["Kernel_Name"]]
    if not writes:
        print("no tree writer dispatch")
        return
    e = writes[-1]
    s = e
    while s > 0 and any(k in rows[s - 1]["Kernel_Name"] for k in ENC):
        s -= 1
        if "tree_size" in rows[s]["Kernel_Name"] and s > 0 and "tree_write" in rows[s - 1]["Kernel_Name"]:
            break  # the previous encode's writers end here
    total, prev = 0.0, None
    for r in rows[s:e + 1]:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (b - a) / 1e3
        total += d
        gap = (a - prev) / 1e3 if prev is not None else 0.0
        prev = b
        grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
        print(f"  {short(r['Kernel_Name']):28s} grid {grid:>9s} {d:9.1f} us  gap {gap:6.1f}")
    wall = (int(rows[e]["End_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1e3
    print(f"  kernels {total:.1f} us, wall {wall:.1f} us")


if __name__ == "__main__":
    main()
