# one GPU call: hub bench + build kernel trace + hub PMC traffic (see profile_bench.sh)
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 > gpurun_out/b_hub1b.json 2> gpurun_out/b_hub1b.err &&
mkdir -p gpurun_out/prof_build1b &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_build1b/kt -o run -- python bench.py --workload build > gpurun_out/prof_build1b/kt.log 2>&1 &&
WORKLOAD=hub STEPS=5 bash tools/profile_bench.sh
