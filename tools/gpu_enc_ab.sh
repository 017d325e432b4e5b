#!/bin/bash
# Encode parity + timings (tools/gpu_encode_quick.sh) and the flat / nested encode write passes'
# LDS counters: bash tools/gpu_enc_ab.sh TAG
set -o pipefail
TAG=${1:-enc}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_encode_quick.sh > $OUT/quick.log 2>&1 || { tail -n 30 $OUT/quick.log; exit 1; }
cat $OUT/quick.log
bash tools/pmc.sh $OUT/pmc "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES" "WRITE_SIZE" -- python3 tools/bench_encode.py > $OUT/pmc.log 2>&1 || { tail -n 20 $OUT/pmc.log; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/pmc/summary.json'))
for k, v in d.items():
    if 'write' in k: print(k, {c: round(x, 1) for c, x in v.items()})
"
