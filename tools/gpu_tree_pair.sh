#!/bin/bash
# Root-group wave groups A/B: tree parity tests, then bench_tree + a kernel trace with the default
# library and each variant given (spec_amd/libspec_amd_<v>.so, e.g. p0 / p4 built with
# -DSPEC_AB_TREE_PAIR=0 / 4).
# Usage (GPU box): bash tools/gpu_tree_pair.sh TAG [variant ...]
set -o pipefail
TAG=${1:-pair}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_specfile.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -n 5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
cp spec_amd/libspec_amd.so /tmp/libspec_amd_default.so
for v in default "$@"; do
  if [ $v != default ]; then cp spec_amd/libspec_amd_$v.so spec_amd/libspec_amd.so; fi
  for i in 1 2; do
    timeout -k 10 300 python tools/bench_tree.py > $OUT/bench_$v$i.json 2> $OUT/bench_$v$i.err || { tail -n 20 $OUT/bench_$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_$v$i.json'))['tree_pkg1']; print('$v', d['decode_ms'], d['encode_ms'], d['bit_exact_and_parity_vs_oracle'])"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_$v -o run -- python3 tools/bench_tree.py > $OUT/prof_$v.log 2>&1 || { tail -n 20 $OUT/prof_$v.log; exit 1; }
  f=$(find $OUT/prof_$v -name "*kernel_trace.csv" | head -n 1); python3 tools/tree_trace.py $f 1 | grep -E "group_0|list_apply|kernels"; python3 tools/tree_enc_trace.py $f | tail -n 6
done
cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so
