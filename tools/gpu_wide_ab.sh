#!/bin/bash
# Wide-schema decode A/B: tests/test_gpu_wide.py, then tools/bench_wide.py with the default
# library and each variant given (spec_amd/libspec_amd_<v>.so), twice each.
# Usage (GPU box): bash tools/gpu_wide_ab.sh TAG variant...
set -o pipefail
TAG=${1:-wab}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_flat.py tests/test_gpu_errors.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
cp spec_amd/libspec_amd.so /tmp/libspec_amd_default.so
for i in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so; else cp spec_amd/libspec_amd_$v.so spec_amd/libspec_amd.so; fi
    timeout -k 10 300 python tools/bench_wide.py > $OUT/w_$v$i.json 2> $OUT/w_$v$i.err || { tail -n 20 $OUT/w_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/w_$v$i.json'))['decode_wide']; print('$v', $i, {k: (x['jit']['ms'], x['jit']['frac'], x['jit_vs_generic_same'], x['oracle_sample_ok']) for k, x in d.items()})"
  done
done
cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so
