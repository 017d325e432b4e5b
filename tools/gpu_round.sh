#!/bin/bash
# One GPU-box pass: parity tests, smoke, PMC traffic (into profiles/pmc_traffic.json, stamped with
# the source revision, so the bench below reports it), bench, rocprofv3 kernel stats + trace.
# Usage (from this container): gpurun --timeout 1100 -- bash tools/gpu_round.sh TAG [quick|full]
set -o pipefail
TAG=${1:-dev}
MODE=${2:-full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -n 3 $OUT/pytest_gpu.log; echo "pytest_rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -n 20 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
if [ "$MODE" != quick ]; then
  echo "== pmc traffic"
  bash tools/pmc.sh $OUT/pmc "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extras > $OUT/pmc.log 2>&1 || { tail -n 20 $OUT/pmc.log; exit 1; }
  python3 tools/pmc_traffic.py $OUT/pmc 1048576 $OUT/pmc_traffic.json > /dev/null && cp $OUT/pmc_traffic.json profiles/pmc_traffic.json && cat $OUT/pmc_traffic.json | head -n 12
fi
echo "== bench"
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -n 20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
[ "$MODE" = quick ] && exit 0
echo "== rocprofv3 stats + trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | head -n 14
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -n 1)
python3 tools/trace_stats.py $f spec_decode_flat_pair_jit 2097152 --json $OUT/decode_flat_1M_trace.json > $OUT/decode_flat_1M_trace.txt && head -n 2 $OUT/decode_flat_1M_trace.txt
# config 5's 2M-record blocks, the flat encoder's passes at 1M records (per-launch-size traces)
python3 tools/trace_stats.py $f spec_decode_flat_pair_jit 4194304 --json $OUT/decode_flat_2M_trace.json > $OUT/decode_flat_2M_trace.txt && head -n 1 $OUT/decode_flat_2M_trace.txt
python3 tools/trace_stats.py $f spec_encode_write_jit 1048576 --json $OUT/encode_write_1M_trace.json > $OUT/encode_write_1M_trace.txt && head -n 1 $OUT/encode_write_1M_trace.txt
python3 tools/trace_stats.py $f spec_encode_size_jit 1048576 --json $OUT/encode_size_1M_trace.json > $OUT/encode_size_1M_trace.txt && head -n 1 $OUT/encode_size_1M_trace.txt
