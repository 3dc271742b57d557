#!/bin/bash
# End-of-round-3 records: the whole GPU suite, then part 2
# (tools/r3_final_b.sh: default bench, hub walk A/B, profiles of $WLS).
set -o pipefail
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/final/tests.txt 2>&1 &&
bash tools/r3_final_b.sh
