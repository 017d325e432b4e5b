#!/bin/bash
# Nested (config 4) parity tests and timing: tests/test_gpu_nested.py, then tools/bench_nested.py.
# Usage: gpurun -- bash tools/gpu_nested.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-nested}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_nested.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_nested.py > $OUT/bench_nested.json 2> $OUT/bench_nested.err || { tail -n 20 $OUT/bench_nested.err; exit 1; }
cat $OUT/bench_nested.json
