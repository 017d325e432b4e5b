#!/bin/bash
# Tree encode + decode leg alone with a kernel trace: the last encode's dispatches and gaps.
set -o pipefail
OUT=gpurun_out/${1:-te}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_tree.py > $OUT/tree.json 2> $OUT/tree.err || { tail -n 20 $OUT/tree.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/tree.json'))['tree_pkg1']; print({k: d[k] for k in ('encode_ms','encode_wall_ms','encode_frac','decode_ms','decode_frac','bit_exact_and_parity_vs_oracle')})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_tree.py > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -n 1); python3 tools/tree_enc_trace.py $f | tee $OUT/enc_trace.txt
python3 tools/tree_trace.py $f 1 | tee $OUT/dec_trace.txt
