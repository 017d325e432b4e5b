#!/bin/bash
# Tree encode per table: the measurement library (spec_amd/libspec_amd_split.so, built
# -DSPEC_AB_TREE_ENC_SPLIT=1) with a kernel trace of tools/bench_tree.py.
# Usage (GPU box): bash tools/gpu_tree_enc_split.sh TAG
set -o pipefail
TAG=${1:-encsplit}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cp spec_amd/libspec_amd_split.so spec_amd/libspec_amd.so
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 tools/bench_tree.py > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -n 1); python3 tools/tree_enc_trace.py $f | tee $OUT/enc_trace.txt
