set -o pipefail
OUT=gpurun_out/tt1; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 tools/bench_tree.py > $OUT/prof.log 2>&1 || { tail -n 20 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -n 1); head -n 1 $f; python3 tools/tree_trace.py $f 1
