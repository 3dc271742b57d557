#!/bin/bash
# The N-GPU bench paths rehearsed with 2 ranks on one GPU over gloo beside the
# 1-GPU run on the same reduced sizes (bio weak scaling with per-rank
# QUERY_1-3 instances, FlyBase / hub strong scaling with the hub's T1 term
# kept split, the build's owner regrouping); tools/rehearse_check.py checks
# the answer sizes.  Chained, each step under its own time limit.
set -o pipefail
mkdir -p gpurun_out/reh
export TMPDIR=/tmp
O=gpurun_out/reh
NB="--no-cpu-baseline --no-materialise"
SMALL="--legs flybase,hub,build --genes 20000 --members 2000000 --bps 5000 --inheritance 10000 --fb-genes 30000 --fb-rows 45000 --hub-links 20000000 --hub-nodes 1000000 --links 20000000 --nodes 1000000 --steps 3 --warmup 1 $NB"
timeout -k 10 300 python bench.py $SMALL > $O/small_1gpu.json 2> $O/small_1gpu.err &&
DAS_SHARD_SMALL=100000 DAS_BENCH_SAME_DEVICE=1 DAS_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 $SMALL \
    > $O/small_2ranks.json 2> $O/small_2ranks.err &&
python tools/rehearse_check.py $O/small_1gpu.json $O/small_2ranks.json $O/rehearse_check.json > /dev/null
