#!/bin/bash
# Round 3, session 16: the GPU suite on HEAD (with the sparse join-build
# variants), smoke, the default bench, the bio step with the dense join build
# and again with the default (A/B).
set -o pipefail
mkdir -p gpurun_out/s16
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise --no-extras"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/s16/tests.txt 2>&1 &&
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s16/smoke.txt 2>&1 &&
timeout -k 10 200 python bench.py > gpurun_out/s16/bench.json 2> gpurun_out/s16/bench.err &&
DAS_DJ_BUILD=dense timeout -k 10 100 python bench.py --workload bio $NB > gpurun_out/s16/bio_dense.json 2> gpurun_out/s16/bio_dense.err &&
timeout -k 10 100 python bench.py --workload bio $NB > gpurun_out/s16/bio_sparse.json 2> gpurun_out/s16/bio_sparse.err
