#!/bin/bash
# Decode timing study on one GPU box: the headline bench twice (run-to-run spread), then an
# interleaved A/B of kernel variants selected by environment variables (tools/ab.py).
# Usage (from this container): gpurun --timeout 900 -- bash tools/gpu_ab.sh TAG 'name=ENV=V,...' ...
set -o pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --no-extras > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -n 20 $OUT/bench_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$i.json')); r=d['roofline']; print('bench', $i, d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['kernel_ms_median'], r['frac'])"
done
if [ $# -gt 0 ]; then
  timeout -k 10 600 python tools/ab.py "$@" --rounds=2 > $OUT/ab.json 2> $OUT/ab.err || { tail -n 20 $OUT/ab.err; exit 1; }
  cat $OUT/ab.json
fi
