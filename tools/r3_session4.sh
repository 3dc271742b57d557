#!/bin/bash
# GPU tests of the changed paths, the default bench (every workload), then
# the 2-rank rehearsal (tools/r3_rehearse.sh).  Chained.
set -o pipefail
mkdir -p gpurun_out/s5
export TMPDIR=/tmp
O=gpurun_out/s5
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "index_join or ij_mid or union or flybase or hub or sharded or semi_join" > $O/tests.txt 2>&1 &&
timeout -k 10 420 python bench.py --steps 10 --warmup 3 > $O/bench_all.json 2> $O/bench_all.err &&
bash tools/r3_rehearse.sh &&
timeout -k 10 200 python tools/host_split.py > gpurun_out/s5/fb_host_split.json 2> gpurun_out/s5/fb_host_split.err
