#!/bin/bash
# Scratch session (run through gpurun): the whole GPU suite, then one bench
# line per workload (no profiler).  Each GPU step has its own time limit and
# the steps are chained, so a failure ends the session.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread --durations=10 > gpurun_out/t_all.txt 2>&1 &&
timeout -k 10 300 python bench.py --workload hub --steps 10 --warmup 3 --no-cpu-baseline --no-materialise > gpurun_out/b_hub.json 2> gpurun_out/b_hub.err &&
timeout -k 10 300 python bench.py --workload build --no-cpu-baseline > gpurun_out/b_build.json 2> gpurun_out/b_build.err &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-materialise > gpurun_out/b_bio.json 2> gpurun_out/b_bio.err &&
timeout -k 10 300 python bench.py --workload flybase --steps 10 --warmup 3 --no-cpu-baseline --no-materialise > gpurun_out/b_flybase.json 2> gpurun_out/b_flybase.err
