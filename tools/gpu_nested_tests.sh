#!/bin/bash
# Nested (config 4) GPU parity tests alone: bash tools/gpu_nested_tests.sh TAG [pytest -k filter]
set -o pipefail
TAG=${1:-nested}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_nested.py ${2:+-k "$2"} -x -v --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "wide|passed|failed|Error" $OUT/pytest.log | tail -15; exit $rc
