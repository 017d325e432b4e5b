#!/bin/bash
# Full GPU suite, then the tree bench leg + a kernel trace of one decode pass, then the headline bench.
# Usage: gpurun -- bash tools/gpu_tree_full.sh TAG
set -o pipefail
TAG=${1:-treefull}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 15 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_tree.py > $OUT/bench_tree.json 2> $OUT/bench_tree.err || { tail -n 20 $OUT/bench_tree.err; exit 1; }
cut -c1-600 $OUT/bench_tree.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 tools/bench_tree.py > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -n 1); python3 tools/tree_trace.py $f 1 | tee $OUT/tree_trace.txt
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -n 20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
