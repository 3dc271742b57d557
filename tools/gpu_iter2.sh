# one GPU call: GPU tests, FlyBase bench + trace, hub (1e9 links) trace
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload flybase --no-cpu-baseline > gpurun_out/b_fly.json 2> gpurun_out/b_fly.err &&
mkdir -p gpurun_out/kt_fly gpurun_out/kt_hub &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_fly -o run -- python bench.py --workload flybase --no-cpu-baseline > gpurun_out/kt_fly/log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_hub -o run -- python bench.py --workload hub --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kt_hub/log 2>&1
