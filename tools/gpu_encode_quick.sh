# Encode parity (flat, nested, golden, C ABI) and encode timings: bash tools/gpu_encode_quick.sh
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_flat.py tests/test_gpu_nested.py tests/test_gpu_golden.py tests/test_gpu_capi.py > gpurun_out/enc_tests.log 2>&1; rc=$?; tail -n 2 gpurun_out/enc_tests.log; [ $rc = 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python3 tools/bench_encode.py || exit 1
  timeout -k 10 300 python3 tools/bench_nested.py | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['nested'])" || exit 1
done
