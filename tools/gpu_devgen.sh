set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_devgen.py > gpurun_out/devgen_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload build > gpurun_out/b_build1b.json 2> gpurun_out/b_build1b.err &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 > gpurun_out/b_hub1b.json 2> gpurun_out/b_hub1b.err &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fullsize.py -k hub > gpurun_out/full_hub.log 2>&1
