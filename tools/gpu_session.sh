set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or hub_join or bio or flybase or composite" > gpurun_out/r2_quick_tests.txt 2>&1 &&
DAS_DJ_VARIANT=0 timeout -k 10 120 python tools/ubench_join.py > gpurun_out/ub_v0.json 2>&1 &&
DAS_DJ_VARIANT=1 timeout -k 10 120 python tools/ubench_join.py > gpurun_out/ub_v1.json 2>&1 &&
DAS_DJ_VARIANT=0 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-materialise > gpurun_out/bio_v0.json 2>/dev/null &&
DAS_DJ_VARIANT=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-materialise > gpurun_out/bio_v1.json 2>/dev/null &&
DAS_HOST_TRACE=1 timeout -k 10 300 python bench.py --workload flybase --steps 3 --warmup 3 --no-cpu-baseline --no-materialise --cprofile gpurun_out/fb_cprofile.txt > gpurun_out/fb_trace.json 2> gpurun_out/fb_trace.err
