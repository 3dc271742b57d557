set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or index_join or flybase or hub or bio" > gpurun_out/tests.txt 2>&1 &&
timeout -k 10 400 python tools/plan_ab.py > gpurun_out/plan_ab.json 2> gpurun_out/plan_ab.err &&
timeout -k 10 300 python bench.py --workload flybase --steps 20 --warmup 3 --no-cpu-baseline --no-materialise > gpurun_out/fb.json 2> gpurun_out/fb.err
