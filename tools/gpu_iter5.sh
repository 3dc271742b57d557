# one GPU call: parity subset, hub (1e9 links) + bio benches, hub trace
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "synthetic or hub or flybase or queries or composite or facade" > gpurun_out/gpu_tests_q.log 2>&1 &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_hub.json 2> gpurun_out/b_hub.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
mkdir -p gpurun_out/kt_hub &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_hub -o run -- python bench.py --workload hub --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/kt_hub/log 2>&1
