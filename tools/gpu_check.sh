#!/bin/bash
# One GPU-box check after a kernel change: the named GPU tests, then the headline bench twice
# (device-resident decode; run-to-run spread), optionally followed by an A/B of env variants.
# Usage (from this container):
#   gpurun --timeout 900 -- bash tools/gpu_check.sh TAG "tests/test_gpu_flat.py ..." ['name=ENV=V,...' ...]
set -o pipefail
TAG=${1:-check}; shift
TESTS=${1:-tests}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 15 $OUT/pytest.log; echo "pytest_rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh $TAG "$@" || exit 1
if [ -n "$PMC" ]; then
  bash tools/pmc.sh $OUT/pmc "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extras > $OUT/pmc.log 2>&1 || { tail -n 20 $OUT/pmc.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/pmc/summary.json')); print(json.dumps({k: v for k, v in d.items() if 'decode' in k}))"
fi
