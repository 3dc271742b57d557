set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "index_join or hub_four or flybase or synthetic" > gpurun_out/ij_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 > gpurun_out/b_hub1b.json 2> gpurun_out/b_hub1b.err &&
timeout -k 10 300 python -u bench.py --workload flybase > gpurun_out/b_fly.json 2> gpurun_out/b_fly.err
