#!/bin/bash
# Flat encode A/B: the encode parity tests with the default library, then tools/bench_encode.py
# alternating the default and each variant (spec_amd/libspec_amd_<v>.so), 3 runs each; then the
# write pass's PMC counters with the default.
# Usage (GPU box): bash tools/gpu_encab.sh TAG "pytest selection" [variant ...]
set -o pipefail
TAG=${1:-encab}; TESTS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
cp spec_amd/libspec_amd.so /tmp/libspec_amd_default.so
for i in 1 2 3; do
  for v in default "$@"; do
    if [ $v = default ]; then cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so; else cp spec_amd/libspec_amd_$v.so spec_amd/libspec_amd.so; fi
    timeout -k 10 300 python3 tools/bench_encode.py > $OUT/e_$v$i.json 2> $OUT/e_$v$i.err || { tail -n 20 $OUT/e_$v$i.err; exit 1; }
    echo "$v $i $(cat $OUT/e_$v$i.json)"
  done
done
cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so
timeout -k 10 300 bash tools/pmc.sh $OUT/pmc "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES" "WRITE_SIZE" "FETCH_SIZE" -- python3 tools/bench_encode.py > $OUT/pmc.log 2>&1 || { tail -n 20 $OUT/pmc.log; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/pmc/summary.json'))
for k, v in d.items():
    if 'encode' in k: print(k, {c: round(x, 1) for c, x in v.items()})
"
