#!/bin/bash
# Headline decode A/B: bench.py's Flat16 decode leg alone (no CPU / extras / verify), alternating
# the default library and each variant given (spec_amd/libspec_amd_<v>.so), 3 runs each.
# Usage (GPU box): bash tools/gpu_headline_ab.sh TAG variant...
set -o pipefail
TAG=${1:-hab}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cp spec_amd/libspec_amd.so /tmp/libspec_amd_default.so
for i in 1 2 3; do
  for v in default "$@"; do
    if [ $v = default ]; then cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so; else cp spec_amd/libspec_amd_$v.so spec_amd/libspec_amd.so; fi
    timeout -k 10 300 python bench.py --no-cpu --no-extras --no-verify --no-native --steps 200 --warmup 30 > $OUT/b_$v$i.json 2> $OUT/b_$v$i.err || { tail -n 20 $OUT/b_$v$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', $i, d['value'], r['kernel_ms_avg'], r['kernel_ms_median'], r['frac'], d['correct'])"
  done
done
cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so
