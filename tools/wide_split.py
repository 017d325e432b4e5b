"""Split tools/prof_wide.sh's wide-kernel launches by schema: bench.wide_leg runs the 40-field
schema's launches first, then (after the generic kernel's) the big-tag schema's, so consecutive
runs of spec_decode_flat_wide_pair_jit dispatches are one schema each.  Writes OUT/wide_split.json:
per segment the median launch time (kernel trace) and the mean of every PMC counter."""
import csv
import glob
import json
import sys
from collections import defaultdict


def segments(rows, key):
    rows = sorted(rows, key=key)
    segs, cur = [], []
    for r in rows:
        if "wide" in r["Kernel_Name"]:
            cur.append(r)
        elif cur:
            segs.append(cur)
            cur = []
    if cur:
        segs.append(cur)
    return [s for s in segs if len(s) > 5]


out = sys.argv[1]
names = ["wide40", "big16"]
res = {n: {} for n in names}
trace = glob.glob(f"{out}/prof/**/*kernel_trace.csv", recursive=True)
if trace:
    for n, s in zip(names, segments(list(csv.DictReader(open(trace[0]))), lambda r: int(r["Start_Timestamp"]))):
        d = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s)
        res[n]["launches"] = len(d)
        res[n]["median_us"] = d[len(d) // 2] / 1e3
for f in sorted(glob.glob(f"{out}/pmc/p*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    disp = defaultdict(list)
    for r in rows:
        disp[int(r["Dispatch_Id"])].append(r)
    heads = [v[0] for v in disp.values()]
    for n, s in zip(names, segments(heads, lambda r: int(r["Dispatch_Id"]))):
        acc = defaultdict(list)
        for h in s:
            for r in disp[int(h["Dispatch_Id"])]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for c, v in acc.items():
            res[n][c] = sum(v) / len(v)
json.dump(res, open(f"{out}/wide_split.json", "w"), indent=1)
print(json.dumps(res, indent=1))
