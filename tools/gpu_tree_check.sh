#!/bin/bash
# Tree GPU tests, then the tree leg with kernel traces (decode pass and encode sets).
# Usage: gpurun --timeout 900 -- bash tools/gpu_tree_check.sh TAG
set -o pipefail
TAG=${1:-tc}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; echo "pytest_rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_tree_enc.sh $TAG/tree_trace > $OUT/trace.log 2>&1 || { tail -n 20 $OUT/trace.log; exit 1; }
head -n 3 $OUT/trace.log; tail -n 12 $OUT/tree_trace/dec_trace.txt
