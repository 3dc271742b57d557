set -o pipefail
mkdir -p gpurun_out/r6h
timeout -k 10 600 python -u -m pytest tests/test_gpu_index_build.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_devgen.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r6h/tests.txt 2>&1 || exit 1
timeout -k 10 700 python bench.py --steps 20 --warmup 5 --detail gpurun_out/r6h/bench_detail.json > gpurun_out/r6h/bench.json 2> gpurun_out/r6h/bench.err || exit 1
