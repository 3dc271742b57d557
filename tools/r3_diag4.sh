#!/bin/bash
# Round-3 session: GPU tests (default = 16-byte output quads in the join
# expansion), then bench A/B of DAS_DJ_QUAD on bio and hub, then the 2-rank
# rehearsal with split terms forced (DAS_SHARD_SMALL) beside 1 GPU.
set -o pipefail
mkdir -p gpurun_out/ab4
export TMPDIR=/tmp
O=gpurun_out/ab4
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 &&
for q in 1 0; do
    DAS_DJ_QUAD=$q timeout -k 10 200 python bench.py --workload bio --steps 20 --warmup 3 $NB > $O/bio_q$q.json 2> $O/bio_q$q.err || exit 12
    DAS_DJ_QUAD=$q timeout -k 10 200 python bench.py --workload hub $NB > $O/hub_q$q.json 2> $O/hub_q$q.err || exit 13
done
SMALL="--legs flybase,hub --genes 20000 --members 2000000 --bps 5000 --inheritance 10000 --fb-genes 30000 --fb-rows 45000 --hub-links 20000000 --hub-nodes 1000000 --steps 3 --warmup 1 $NB" &&
timeout -k 10 300 python bench.py $SMALL > $O/small_1gpu.json 2> $O/small_1gpu.err &&
DAS_SHARD_SMALL=100000 DAS_BENCH_SAME_DEVICE=1 DAS_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 $SMALL \
    > $O/small_2ranks.json 2> $O/small_2ranks.err
