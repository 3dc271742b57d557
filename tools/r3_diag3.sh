#!/bin/bash
# Round-3 A/B session (gpurun from the repo root):
#   1. hub flag-pass variants DAS_FILT_OPT=0..3
#   2. bio with scan views at every size (DAS_SCAN_VIEWS=1) vs the default
#   3. the N-GPU bench path rehearsed with 2 ranks on one GPU (gloo) beside
#      the 1-GPU run of the same reduced FlyBase / hub KBs: per-query counts
#      must agree
# Each step under its own time limit, chained.
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
O=gpurun_out/ab
NB="--no-cpu-baseline --no-materialise"
for opt in 0 1 2 3; do
    DAS_FILT_OPT=$opt timeout -k 10 200 python bench.py --workload hub $NB > $O/hub_opt$opt.json 2> $O/hub_opt$opt.err || exit 11
done
timeout -k 10 200 python bench.py --workload bio --steps 20 --warmup 3 $NB > $O/bio_default.json 2> $O/bio_default.err &&
DAS_SCAN_VIEWS=1 timeout -k 10 200 python bench.py --workload bio --steps 20 --warmup 3 $NB > $O/bio_views.json 2> $O/bio_views.err &&
SMALL="--legs flybase,hub --genes 20000 --members 2000000 --bps 5000 --inheritance 10000 --fb-genes 30000 --fb-rows 45000 --hub-links 20000000 --hub-nodes 1000000 --steps 3 --warmup 1 $NB" &&
timeout -k 10 300 python bench.py $SMALL > $O/small_1gpu.json 2> $O/small_1gpu.err &&
DAS_BENCH_SAME_DEVICE=1 DAS_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 $SMALL \
    > $O/small_2ranks.json 2> $O/small_2ranks.err
