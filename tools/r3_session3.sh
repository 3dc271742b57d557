#!/bin/bash
# GPU tests of the paths changed since the last full run, the FlyBase bench,
# then rocprof profiles (bio, hub) and the hub chunk-size A/B.  Chained, each
# step under its own time limit.
set -o pipefail
mkdir -p gpurun_out/s4
export TMPDIR=/tmp
O=gpurun_out/s4
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "index_join or ij_mid or union or flybase or plan_cache or golden or chain or hub" > $O/tests.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload flybase --steps 20 --warmup 3 $NB > $O/fb.json 2> $O/fb.err &&
WLS="${WLS:-bio hub}" CHUNK_AB=${CHUNK_AB:-1} bash tools/r3_profiles.sh
