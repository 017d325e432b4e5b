set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/icache
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d gpurun_out/icache/p1 -o run -- python3 tools/bench_tree.py > gpurun_out/icache/p1.log 2>&1 || { tail -n 5 gpurun_out/icache/p1.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/icache | grep -A4 "group_0p2\|write_set\|group_set\|size_set"
