set -o pipefail
OUT=gpurun_out/${1:-wide}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tree.py -x -v --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "wide|passed|failed|Error" $OUT/pytest.log | tail -15; exit $rc
