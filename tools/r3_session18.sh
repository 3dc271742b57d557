#!/bin/bash
# Round 3, session 18: the GPU suite on HEAD (sparse join build and fused
# guard by default), then the bio step.
set -o pipefail
mkdir -p gpurun_out/s18
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise --no-extras"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/s18/tests.txt 2>&1 &&
timeout -k 10 100 python bench.py --workload bio $NB > gpurun_out/s18/bio.json 2> gpurun_out/s18/bio.err
