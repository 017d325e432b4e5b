#!/bin/bash
# Round evidence in one GPU call: tools/gpu_round.sh (tests, smoke, PMC traffic, bench, kernel
# stats + trace), then the nested and tree kernel stats + PMC passes.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_round_all.sh TAG
set -o pipefail
TAG=${1:-round}
bash tools/gpu_round.sh $TAG full || exit $?
echo "== nested prof"
bash tools/prof_nested.sh gpurun_out/$TAG/nested > gpurun_out/$TAG/nested.log 2>&1 || { tail -n 20 gpurun_out/$TAG/nested.log; exit 1; }
echo "== tree prof"
bash tools/prof_tree.sh gpurun_out/$TAG/tree > gpurun_out/$TAG/tree.log 2>&1 || { tail -n 20 gpurun_out/$TAG/tree.log; exit 1; }
echo "== wide prof"
bash tools/prof_wide.sh gpurun_out/$TAG/wide > gpurun_out/$TAG/wide.log 2>&1 && python3 tools/wide_split.py gpurun_out/$TAG/wide > /dev/null || { tail -n 20 gpurun_out/$TAG/wide.log; exit 1; }
echo "== tree encode/decode trace"
bash tools/gpu_tree_enc.sh $TAG/tree_trace > gpurun_out/$TAG/tree_trace.log 2>&1 || { tail -n 20 gpurun_out/$TAG/tree_trace.log; exit 1; }
tail -n 3 gpurun_out/$TAG/tree_trace/enc_trace.txt
echo done
