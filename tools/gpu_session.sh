# scratch GPU session (edited per experiment); every step bounded and chained
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-materialise"
timeout -k 10 600 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.txt 2>&1 &&
for v in 1 0 1 0; do DAS_DJ_FIXED=$v timeout -k 10 200 $B > gpurun_out/bio_fixed$v.json 2>/dev/null && tail -n 1 gpurun_out/bio_fixed$v.json >> gpurun_out/ab.jsonl || exit 1; done &&
timeout -k 10 300 $B --workload flybase > gpurun_out/fb_plan.json 2> gpurun_out/fb_plan.err &&
DAS_PLAN=0 timeout -k 10 300 $B --workload flybase > gpurun_out/fb_host.json 2> gpurun_out/fb_host.err
