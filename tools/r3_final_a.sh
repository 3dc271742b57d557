#!/bin/bash
# End-of-round-3 records, part 1: the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/final/tests.txt 2>&1
