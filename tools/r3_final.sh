#!/bin/bash
# End-of-round-3 records: the whole GPU suite, the default bench (every
# workload), rocprof profiles of the workloads named in $WLS, then the hub
# walk A/B (software-pipelined one walk, DAS_FILT_PIPE=1).
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/final/tests.txt 2>&1 &&
timeout -k 10 500 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err &&
for w in ${WLS:-}; do
    TAG=r3f WORKLOAD=$w bash tools/profile_bench.sh || exit 20
done &&
DAS_FILT_PIPE=1 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/final/hub_pipe.json 2> gpurun_out/final/hub_pipe.err &&
timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/final/hub_walk.json 2> gpurun_out/final/hub_walk.err
