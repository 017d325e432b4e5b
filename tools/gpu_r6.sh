#!/bin/bash
# Round-6 check in one GPU call: the GPU test suite (or the named tests), smoke, a short bench.
# Usage: gpurun --timeout 900 -- bash tools/gpu_r6.sh TAG ["tests ..."]
set -o pipefail
TAG=${1:-r6}; TESTS=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 8 $OUT/pytest.log; echo "pytest_rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -n 20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d[k] for k in ('value','ms_per_step')}, d['roofline']['frac'])"
