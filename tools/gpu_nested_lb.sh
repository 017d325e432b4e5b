set -o pipefail
OUT=gpurun_out/nlb; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_nested.py > $OUT/t_default.log 2>&1; tail -1 $OUT/t_default.log
for i in 1 2; do timeout -k 10 300 python3 tools/bench_nested.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['nested']; print('default', d['onepass_ms'], d['twopass_ms'])" || exit 1; done
cp spec_amd/libspec_amd_lb.so spec_amd/libspec_amd.so
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_nested.py > $OUT/t_lb.log 2>&1; tail -1 $OUT/t_lb.log
for i in 1 2; do timeout -k 10 300 python3 tools/bench_nested.py | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['nested']; print('lookback', d['onepass_ms'], d['twopass_ms'])" || exit 1; done
