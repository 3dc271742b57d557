#!/bin/bash
# End-of-round-3 records, part 2: the default bench (every workload), the
# hub walk A/B (DAS_FILT_PIPE=1), then rocprof profiles of $WLS.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 500 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err &&
DAS_FILT_PIPE=1 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/final/hub_pipe.json 2> gpurun_out/final/hub_pipe.err &&
timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/final/hub_walk.json 2> gpurun_out/final/hub_walk.err &&
for w in ${WLS:-}; do
    TAG=r3f WORKLOAD=$w bash tools/profile_bench.sh || exit 20
done
