#!/bin/bash
# GPU tests touching index joins / FlyBase / plan cache, then the FlyBase
# bench A/B of the one-launch mid-size index join (DAS_IJ_MID), then r3
# profiles of bio and hub (tools/profile_bench.sh).  Chained, each step
# under its own time limit.
set -o pipefail
mkdir -p gpurun_out/s2
export TMPDIR=/tmp
O=gpurun_out/s2
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "index_join or ij_mid or flybase or plan_cache or golden or chain" > $O/tests.txt 2>&1 &&
DAS_IJ_MID=1 timeout -k 10 200 python bench.py --workload flybase --steps 20 --warmup 3 $NB > $O/fb_mid1.json 2> $O/fb_mid1.err &&
DAS_IJ_MID=0 timeout -k 10 200 python bench.py --workload flybase --steps 20 --warmup 3 $NB > $O/fb_mid0.json 2> $O/fb_mid0.err &&
TAG=r3 WORKLOAD=bio bash tools/profile_bench.sh && TAG=r3 WORKLOAD=hub bash tools/profile_bench.sh
