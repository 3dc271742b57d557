set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 > gpurun_out/b_hub1b.json 2> gpurun_out/b_hub1b.err &&
timeout -k 10 300 python -u bench.py --workload flybase > gpurun_out/b_fly.json 2> gpurun_out/b_fly.err
