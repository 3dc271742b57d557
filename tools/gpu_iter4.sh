# one GPU call: all GPU tests, hub (1e9 links) + bio + FlyBase benches, hub trace
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_hub.json 2> gpurun_out/b_hub.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
timeout -k 10 300 python -u bench.py --workload flybase --no-cpu-baseline > gpurun_out/b_fly.json 2> gpurun_out/b_fly.err &&
mkdir -p gpurun_out/kt_hub &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_hub -o run -- python bench.py --workload hub --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kt_hub/log 2>&1
