#!/usr/bin/env python3
"""The dispatches of the last spec_tree_decoder_run pass in a rocprofv3 kernel trace (csv), in
launch order: kernel, grid, duration.  A pass starts with the records' group kernel.

Usage: python3 tools/tree_trace.py RUN_kernel_trace.csv [PASSES]
"""
import csv
import sys


def short(name):
    name = name.replace("(anonymous namespace)", "anon")
    return name.split("(")[0].split("::")[-1]


DECODE = ("spec_tree_group", "list_tiles_kernel", "list_top_kernel", "list_apply_kernel", "rows_out_kernel",
          "tree_group_kernel", "tree_rows")


def is_root(name):
    """The records' group kernel, which starts a pass (spec_tree_group_0 / spec_tree_group_0pP)."""
    s = short(name)
    return s == "spec_tree_group_0" or (s.startswith("spec_tree_group_0p") and s[18:].isdigit())


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a pass: from a records' group launch through the decode launches that follow it (rows_out_kernel
    # ended a pass until round 6; the pass's last list scan now writes rows_out itself)
    starts = [i for i, r in enumerate(rows) if is_root(r["Kernel_Name"])]
    spans = []
    for s0 in starts:
        e = s0
        while e + 1 < len(rows) and not is_root(rows[e + 1]["Kernel_Name"]) and \
                any(k in rows[e + 1]["Kernel_Name"] for k in DECODE):
            e += 1
        spans.append((s0, e))
    if not spans:
        print("no pass found")
        return
    for k in range(min(passes, len(spans))):
        s, e = spans[-1 - k]
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
