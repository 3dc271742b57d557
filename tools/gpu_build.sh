# one GPU call: build-path parity subset, 1e9-link build bench, build kernel trace (timestamps kept)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_devgen.py tests/test_gpu_parity.py -k "devgen or build or reference_atoms or synthetic_matches or hub_four or incoming or keyspace or loader" > gpurun_out/gpu_tests_build.log 2>&1 &&
DAS_ALLOC_TRACE=1 timeout -k 10 300 python -u bench.py --workload build > gpurun_out/b_build.json 2> gpurun_out/b_build.err &&
mkdir -p gpurun_out/kt_build &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_build -o run -- python bench.py --workload build > gpurun_out/kt_build/log 2>&1
