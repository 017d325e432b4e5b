set -o pipefail
OUT=gpurun_out/enc1; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_nested.py tests/test_gpu_flat.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_nested.py > $OUT/bench_nested.json 2> $OUT/bench_nested.err || { tail -n 20 $OUT/bench_nested.err; exit 1; }
python3 -c "import json; print(json.load(open('$OUT/bench_nested.json'))['nested'])"
timeout -k 10 300 python bench.py --no-cpu --steps 50 > $OUT/bench.json 2> $OUT/bench.err || { tail -n 20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['encode'], d['nested']['encode_ms'])"
