#!/bin/bash
# Tree path on the GPU box: parity tests, the tree bench leg, a kernel trace of one decode pass.
# Usage: gpurun -- bash tools/gpu_tree.sh TAG [tests-filter]
set -o pipefail
TAG=${1:-tree}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py ${2:+-k "$2"} -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_tree.py > $OUT/bench_tree.json 2> $OUT/bench_tree.err || { tail -n 20 $OUT/bench_tree.err; exit 1; }
cat $OUT/bench_tree.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 tools/bench_tree.py > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -n 1); python3 tools/tree_trace.py $f 1
