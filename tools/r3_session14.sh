#!/bin/bash
# Round 3, session 14: the default bench (every workload) after the in-place
# join-build descriptors, then the bio rocprof profile (kernel stats, PMC
# traffic, roofline check) of the same code.
set -o pipefail
mkdir -p gpurun_out/s14
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/s14/bench.json 2> gpurun_out/s14/bench.err &&
TAG=r3g WORKLOAD=bio bash tools/profile_bench.sh
[ $? -eq 0 ] && DAS_TRACE=1 timeout -k 10 200 python tools/trace_plan.py --workload bio > gpurun_out/s14/bio_trace.out 2> gpurun_out/s14/bio_trace.txt
