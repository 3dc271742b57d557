#!/bin/bash
# Scratch session (run through gpurun): the whole GPU suite, then one bench
# line per workload (no profiler).  Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=10 > gpurun_out/t_all.txt 2>&1 &&
for w in hub bio flybase build; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-materialise > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit 1
done
