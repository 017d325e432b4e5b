#!/bin/bash
# Kernel stats (rocprofv3 --kernel-trace --stats) and optionally the standard PMC passes of one
# command.  Usage (GPU box): bash tools/prof.sh OUTDIR [pmc] -- cmd args
set -o pipefail
OUT=$1; shift
PMC=0
if [ "$1" = "pmc" ]; then PMC=1; shift; fi
[ "$1" = "--" ] && shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- "$@" > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | head -n 16
[ $PMC = 1 ] || exit 0
bash tools/pmc.sh $OUT/pmc "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY" -- "$@" > $OUT/pmc.log 2>&1 || { tail -n 20 $OUT/pmc.log; exit 1; }
tail -n 60 $OUT/pmc.log
