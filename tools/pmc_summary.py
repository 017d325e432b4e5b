"""Summarise rocprofv3 --pmc CSVs: per kernel name, mean of each counter over dispatches."""
import csv
import glob
import json
import sys
from collections import defaultdict

out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{out}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        if "spec" not in name:
            continue
        short = name.replace("(anonymous namespace)", "anon").split("(")[0][-60:]
        acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}
json.dump(res, open(f"{out}/summary.json", "w"), indent=1)
for k, d in res.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:16.1f}")
