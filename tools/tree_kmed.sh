#!/bin/bash
# Per-kernel median durations of tools/bench_tree.py (pkg1 tree decode + encode) under a kernel
# trace, plus the leg's event-timed decode/encode.  Usage (GPU box): bash tools/tree_kmed.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/tkm}; mkdir -p $OUT; export TMPDIR=/tmp
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 tools/bench_tree.py > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -n 1)
python3 - $f <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0].split("::")[-1]
    if "tree" in n or "list_" in n or "scan" in n or "rows_out" in n:
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items()):
    v.sort(); print(f"  {n:24s} {len(v):5d} {v[len(v)//2]:8.1f} us")
PY
grep -o '"decode_ms": [0-9.]*\|"encode_ms": [0-9.]*\|"bit_exact_and_parity_vs_oracle": [a-z]*' $OUT/prof.log | tr '\n' ' '; echo
