#!/bin/bash
# Native multi-device path on one GPU box: its parity tests, then the bench's native_shard leg
# at N=1 (RCCL communicator forced: gather = send to self) and in a 2-rank gloo rehearsal
# (two shards sharing the GPU).  Usage: gpurun -- bash tools/gpu_native.sh TAG
set -o pipefail
TAG=${1:-native}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== native shard tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_native.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -n 40; [ $rc -eq 0 ] || exit $rc
echo "== bench N=1"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -n 30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['correct']); print(json.dumps(d.get('native_shard')))"
echo "== bench --gpus 2 gloo rehearsal"
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --no-cpu > $OUT/bench_gpus2.json 2> $OUT/bench_gpus2.err || { tail -n 30 $OUT/bench_gpus2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_gpus2.json')); print(d['value'], d['correct']); print(json.dumps(d.get('native_shard')))"
