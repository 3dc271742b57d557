# one GPU call: join-path parity subset, full-size properties, bio/hub benches, bio kernel trace
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "synthetic or hub or index_join or flybase or composite or queries" > gpurun_out/gpu_tests_q.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fullsize.py > gpurun_out/gpu_full.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_hub.json 2> gpurun_out/b_hub.err &&
mkdir -p gpurun_out/kt_bio &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_bio -o run -- python bench.py --no-cpu-baseline > gpurun_out/kt_bio/log 2>&1
