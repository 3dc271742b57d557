#!/bin/bash
# The config-4 build's N-GPU path (hash owners, regroup rows on their owners
# by all-to-all, build the shard) rehearsed with 2 ranks on one GPU over gloo,
# beside the 1-GPU build of the same generated KB: the distinct links
# indexed must agree (each link indexed exactly once, on its owner).
set -o pipefail
mkdir -p gpurun_out/rb
export TMPDIR=/tmp
O=gpurun_out/rb
A="--workload build --links 20000000 --nodes 1000000 --no-cpu-baseline"
timeout -k 10 200 python bench.py $A > $O/build_1gpu.json 2> $O/build_1gpu.err &&
DAS_BENCH_SAME_DEVICE=1 DAS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 $A \
    > $O/build_2ranks.json 2> $O/build_2ranks.err
