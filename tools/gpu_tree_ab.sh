#!/bin/bash
# Tree encode A/B: tools/bench_tree.py alternating the default library and each variant
# (spec_amd/libspec_amd_<v>.so, tools/build_tree_variant.sh), 3 runs each.
# Usage (GPU box): bash tools/gpu_tree_ab.sh TAG [variant ...]
set -o pipefail
TAG=${1:-treeab}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cp spec_amd/libspec_amd.so /tmp/libspec_amd_default.so
for i in 1 2 3; do
  for v in default "$@"; do
    if [ $v = default ]; then cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so; else cp spec_amd/libspec_amd_$v.so spec_amd/libspec_amd.so; fi
    timeout -k 10 300 python3 tools/bench_tree.py > $OUT/t_$v$i.json 2> $OUT/t_$v$i.err || { tail -n 20 $OUT/t_$v$i.err; cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/t_$v$i.json'))['tree_pkg1']; print('$v $i', {k: d[k] for k in ('encode_ms','decode_ms','bit_exact_and_parity_vs_oracle')})"
  done
done
cp /tmp/libspec_amd_default.so spec_amd/libspec_amd.so
