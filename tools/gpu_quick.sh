#!/bin/bash
# A subset of the GPU tests (pytest -k expression or files), then optionally a short bench.
# Usage: gpurun -- bash tools/gpu_quick.sh TAG "pytest args" [bench]
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest $2"
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $2 > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -n 60; [ $rc -eq 0 ] || exit $rc
if [ "$3" = bench ]; then
  echo "== bench"
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -n 30 $OUT/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['correct'], d['checks']); print(json.dumps(d.get('native_shard'))); print(json.dumps(d.get('tree_pkg1')))"
fi
