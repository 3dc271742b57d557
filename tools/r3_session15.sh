#!/bin/bash
# Round 3, session 15 (sessions 13 + 14 in one call): the GPU suite on HEAD
# (with the sparse join-build variant), smoke, the bio step with the dense
# join build (A/B), the default bench (every workload), the bio rocprof
# profile, a bio plan trace.
set -o pipefail
mkdir -p gpurun_out/s15
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise --no-extras"
timeout -k 10 560 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/s15/tests.txt 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s15/smoke.txt 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/s15/bench.json 2> gpurun_out/s15/bench.err &&
DAS_DJ_BUILD=dense timeout -k 10 120 python bench.py --workload bio $NB > gpurun_out/s15/bio_dense.json 2> gpurun_out/s15/bio_dense.err &&
timeout -k 10 120 python bench.py --workload bio $NB > gpurun_out/s15/bio_sparse.json 2> gpurun_out/s15/bio_sparse.err &&
BENCH_TIMEOUT=150 PROF_TIMEOUT=120 TAG=r3g WORKLOAD=bio bash tools/profile_bench.sh &&
DAS_TRACE=1 timeout -k 10 120 python tools/trace_plan.py --workload bio > gpurun_out/s15/bio_trace.out 2> gpurun_out/s15/bio_trace.txt
