#!/bin/bash
# End-of-round-3 records, part 2: the default bench (every workload), the
# hub walk A/B (DAS_FILT_PIPE=1 / DAS_FILT_LOOKBACK=1 after their parity
# cases), then rocprof profiles of $WLS.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 500 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err &&
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
    -k "semi_join_multi" > gpurun_out/final/tests_walk.txt 2>&1 &&
DAS_FILT_PIPE=1 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/final/hub_pipe.json 2> gpurun_out/final/hub_pipe.err &&
DAS_FILT_LOOKBACK=1 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/final/hub_lookback.json 2> gpurun_out/final/hub_lookback.err &&
timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/final/hub_walk.json 2> gpurun_out/final/hub_walk.err &&
for w in ${WLS:-}; do
    TAG=r3f WORKLOAD=$w bash tools/profile_bench.sh || exit 20
done
