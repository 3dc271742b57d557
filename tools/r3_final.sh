#!/bin/bash
# End-of-round-3 records: the whole GPU suite, the default bench (every
# workload), then rocprof profiles of the workloads named in $WLS.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/final/tests.txt 2>&1 &&
timeout -k 10 500 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err &&
for w in ${WLS:-}; do
    TAG=r3f WORKLOAD=$w bash tools/profile_bench.sh || exit 20
done
