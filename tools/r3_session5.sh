#!/bin/bash
# Sharded GPU tests (incl. QUERY_1-3 shapes), the 2-rank rehearsal with its
# check, the hub A/B (chunk size, flag-pass unroll), then the bio profile.
set -o pipefail
mkdir -p gpurun_out/s6
export TMPDIR=/tmp
O=gpurun_out/s6
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "sharded or golden" > $O/tests.txt 2>&1 &&
bash tools/r3_rehearse.sh &&
bash tools/r3_hub_chunk.sh &&
TAG=r3 WORKLOAD=bio bash tools/profile_bench.sh
