#!/bin/bash
# Wave-pair decode checks: the flat (incl. *Err masks), wide, golden and nested GPU parity tests,
# then the nested decode A/B (tools/gpu_nenc_ab.sh) against the variants given.
# Usage (GPU box): bash tools/gpu_pair_tests.sh TAG [variant ...]
set -o pipefail
TAG=${1:-pair}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_errors.py tests/test_gpu_flat.py tests/test_gpu_wide.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_flat.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_flat.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_nenc_ab.sh $TAG "$@"
