set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nested.py > gpurun_out/nc_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/nc_tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 300 python3 tools/bench_nested.py || exit 1; done
