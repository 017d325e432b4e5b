set -o pipefail
mkdir -p gpurun_out/reh; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --no-cpu > gpurun_out/reh/bench_gpus2_gloo.json 2> gpurun_out/reh/err.log || { tail -n 30 gpurun_out/reh/err.log; exit 1; }
cut -c1-700 gpurun_out/reh/bench_gpus2_gloo.json
