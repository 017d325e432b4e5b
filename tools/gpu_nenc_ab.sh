#!/bin/bash
# Nested encode A/B: nested parity tests with the default library, then tools/bench_nested.py
# with it and with each variant given (spec_amd/libspec_amd_<v>.so).
# Usage (GPU box): bash tools/gpu_nenc_ab.sh TAG [variant ...]
set -o pipefail
TAG=${1:-nenc}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_nested.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
cp spec_amd/libspec_amd.so /tmp/libspec_amd_default.so
for v in default "$@"; do
  if [ $v != default ]; then cp spec_amd/libspec_amd_$v.so spec_amd/libspec_amd.so; fi
  for i in 1 2; do
    timeout -k 10 300 python3 tools/bench_nested.py > $OUT/bench_$v$i.json 2> $OUT/bench_$v$i.err || { tail -n 20 $OUT/bench_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_$v$i.json'))['nested']; print('$v', 'enc', d['encode_ms'], 'dec', d['onepass_ms'], d['twopass_ms'], d.get('ok'))"
  done
done
cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so
