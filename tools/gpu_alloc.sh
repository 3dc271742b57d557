set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
DAS_ALLOC_TRACE=1 timeout -k 10 300 python -u bench.py --workload build > gpurun_out/b_build1b.json 2> gpurun_out/b_build1b.err &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 > gpurun_out/b_hub1b.json 2> gpurun_out/b_hub1b.err &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1
