#!/bin/bash
# Sparse key directories (one load per index-join probe instead of a binary
# search) and the one-walk filtered expansion (DAS_FILT_LOCAL=1): parity
# tests, hub / FlyBase A/B, bio plan trace.
set -o pipefail
mkdir -p gpurun_out/s10
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    -k "semi_join_multi or hub or index_join" > gpurun_out/s10/tests1.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s10/hub_sparse.json 2> gpurun_out/s10/hub_sparse.err &&
DAS_KEY_DIR_SPARSE=0 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s10/hub_dense.json 2> gpurun_out/s10/hub_dense.err &&
DAS_FILT_LOCAL=1 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s10/hub_sparse_local.json 2> gpurun_out/s10/hub_sparse_local.err &&
timeout -k 10 200 python bench.py --workload flybase --steps 20 --warmup 3 $NB > gpurun_out/s10/fb_sparse.json 2> gpurun_out/s10/fb_sparse.err &&
DAS_KEY_DIR_SPARSE=0 timeout -k 10 200 python bench.py --workload flybase --steps 20 --warmup 3 $NB > gpurun_out/s10/fb_dense.json 2> gpurun_out/s10/fb_dense.err &&
DAS_TRACE=1 timeout -k 10 200 python tools/trace_plan.py --workload bio > gpurun_out/s10/bio_trace.out 2> gpurun_out/s10/bio_trace.txt &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "flybase or golden" > gpurun_out/s10/tests2.txt 2>&1
