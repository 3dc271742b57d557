#!/bin/bash
# Scratch session (run through gpurun): FlyBase host profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload flybase --steps 20 --warmup 3 --no-cpu-baseline --no-materialise --cprofile gpurun_out/fb_cprofile.txt > gpurun_out/fb_cp.json 2> gpurun_out/fb_cp.err &&
timeout -k 10 300 python tools/host_split.py > gpurun_out/host_split.json 2> gpurun_out/host_split.err &&
DAS_TRACE=1 timeout -k 10 300 python tools/trace_plan.py > gpurun_out/trace_plan.out 2> gpurun_out/trace_plan.txt
