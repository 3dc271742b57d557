# one GPU call: full GPU test suite, default bench (config 2 bio), kernel trace + PMC traffic
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
WORKLOAD=bio STEPS=10 bash tools/profile_bench.sh
