#!/bin/bash
# One GPU session (run through gpurun from the repo root): the GPU parity
# suite, then the bench + rocprof + PMC passes of the workloads named in
# WORKLOADS (default: bio).  Steps are chained with &&, each under its own
# time limit, so a failure ends the session.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run_tests() {
    timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 150 \
        --timeout-method thread --durations=15 > gpurun_out/tests.txt 2>&1
}
run_profiles() {
    for w in ${WORKLOADS:-bio}; do
        WORKLOAD=$w bash tools/profile_bench.sh || return 1
    done
}
if [ "${SKIP_TESTS:-0}" = "1" ]; then run_profiles; else run_tests && run_profiles; fi
