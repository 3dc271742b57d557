# one GPU call: all GPU tests, hub (1e9 links) + bio + build (1e9) benches, hub trace
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_hub.json 2> gpurun_out/b_hub.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
timeout -k 10 300 python -u bench.py --workload build > gpurun_out/b_build.json 2> gpurun_out/b_build.err &&
mkdir -p gpurun_out/kt_hub gpurun_out/kt_build &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_hub -o run -- python bench.py --workload hub --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kt_hub/log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_build -o run -- python bench.py --workload build > gpurun_out/kt_build/log 2>&1
