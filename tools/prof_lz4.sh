#!/bin/bash
# LZ4 leg (tools/bench_lz4.py): rocprofv3 kernel stats + PMC passes; prints the LZ4 kernels' counters.
# Usage (GPU box): bash tools/prof_lz4.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/lz4}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_lz4.py > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | head -n 8
bash tools/pmc.sh $OUT/pmc "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM" -- python3 tools/bench_lz4.py > $OUT/pmc.log 2>&1 || { tail -n 20 $OUT/pmc.log; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/pmc/summary.json'))
for k, v in d.items():
    if 'lz4' in k: print(k[:60], json.dumps({c: round(x) for c, x in v.items()}))
"
