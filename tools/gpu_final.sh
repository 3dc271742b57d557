# one GPU call: full GPU suite, smoke, default bench (config 2 bio), build bench (config 4)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
timeout -k 10 300 python -u bench.py --workload build > gpurun_out/b_build.json 2> gpurun_out/b_build.err &&
timeout -k 10 300 python -u bench.py --workload flybase --no-cpu-baseline > gpurun_out/b_flybase.json 2> gpurun_out/b_flybase.err
