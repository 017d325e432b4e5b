#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only — no sys/runtime trace).
# Usage: bash tools/pmc.sh OUTDIR "counter group 1" "counter group 2" ... -- cmd args
set -o pipefail
OUT=$1; shift
groups=()
while [ "$1" != "--" ]; do groups+=("$1"); shift; done
shift
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p $OUT
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $g --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -n 20 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT
