#!/bin/bash
# The 8-rank flow the driver's SCALE run executes (bench.py --gpus 8: 8 rank processes plus the
# native one-process child driving 8 shards), rehearsed on a one-GPU box: every rank on cuda:0
# over gloo, the native child's 8 shards sharing the GPU.  Wall time recorded.
# Usage: gpurun --timeout 900 -- bash tools/gpu_rehearsal8.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-reh8}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
t0=$(date +%s.%N)
timeout -k 10 800 python bench.py --gpus 8 --backend gloo "$@" > $OUT/bench_gpus8_gloo.json 2> $OUT/err.log
rc=$?
t1=$(date +%s.%N)
python3 -c "print('wall_s', round($t1 - $t0, 1))" | tee $OUT/wall.txt
[ $rc -eq 0 ] || { tail -n 30 $OUT/err.log; exit $rc; }
cut -c1-900 $OUT/bench_gpus8_gloo.json
