#!/bin/bash
# Semi-join duplicate flag read back with the count (one read-back per
# semi-join), one flag read-back per key-set intersection: parity tests of
# every semi-join user, then the default bench (every workload).
set -o pipefail
mkdir -p gpurun_out/s13
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "golden or semi or hub or bio or reference or template or flybase or sharded" > gpurun_out/s13/tests.txt 2>&1 &&
timeout -k 10 500 python bench.py > gpurun_out/s13/bench.json 2> gpurun_out/s13/bench.err &&
true
[ $? -eq 0 ] && KERNEL='k_dj_filt<2|k_dj_write_bal|k_chunk_compact' WORKLOAD=hub bash tools/pmc_kernel.sh
