set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread --durations=10 > gpurun_out/tests.txt 2>&1 &&
timeout -k 10 400 python tools/plan_ab.py > gpurun_out/plan_ab.json 2> gpurun_out/plan_ab.err &&
timeout -k 10 300 python bench.py --workload flybase --steps 20 --warmup 3 --no-cpu-baseline --no-materialise > gpurun_out/fb.json 2> gpurun_out/fb.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-materialise > gpurun_out/bio.json 2> gpurun_out/bio.err
