#!/bin/bash
# Nested (config 4) and tree (pkg1) kernel stats + PMC passes.  Usage: gpurun -- bash tools/gpu_profiles.sh TAG
set -o pipefail
TAG=${1:-prof}
mkdir -p gpurun_out/$TAG
bash tools/prof_nested.sh gpurun_out/$TAG/nested > gpurun_out/$TAG/nested.log 2>&1 || { tail -n 20 gpurun_out/$TAG/nested.log; exit 1; }
bash tools/prof_tree.sh gpurun_out/$TAG/tree > gpurun_out/$TAG/tree.log 2>&1 || { tail -n 20 gpurun_out/$TAG/tree.log; exit 1; }
echo done
