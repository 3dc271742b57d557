# one GPU call: bio bench with dominant-kernel events vs every-scope events, hub bench, bio kernel trace
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
timeout -k 10 300 python -u bench.py --events all --no-cpu-baseline > gpurun_out/b_bio_all.json 2> gpurun_out/b_bio_all.err &&
timeout -k 10 300 python -u bench.py --workload flybase --no-cpu-baseline > gpurun_out/b_flybase.json 2> gpurun_out/b_flybase.err &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 > gpurun_out/b_hub.json 2> gpurun_out/b_hub.err &&
mkdir -p gpurun_out/kt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/kt/log 2>&1
