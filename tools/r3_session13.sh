#!/bin/bash
# Round 3, session 13: the whole GPU suite on HEAD (with the sparse join-build
# variant), smoke, then the bio step A/B of the join build (slot arrays vs
# descriptors written in place).
set -o pipefail
mkdir -p gpurun_out/s13
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise --no-extras"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/s13/tests.txt 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s13/smoke.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload bio $NB > gpurun_out/s13/bio_sparse.json 2> gpurun_out/s13/bio_sparse.err &&
DAS_DJ_BUILD=dense timeout -k 10 200 python bench.py --workload bio $NB > gpurun_out/s13/bio_dense.json 2> gpurun_out/s13/bio_dense.err &&
timeout -k 10 200 python bench.py --workload bio $NB > gpurun_out/s13/bio_sparse2.json 2> gpurun_out/s13/bio_sparse2.err
