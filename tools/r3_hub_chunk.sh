#!/bin/bash
# Hub filtered-expansion A/B: chunk size (DAS_FILT_CHUNK 1024 / 2048 / 4096)
# and the flag pass's unroll depth (DAS_FILT_UNROLL 8 / 16 at 1024).
set -o pipefail
mkdir -p gpurun_out/s3
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
for ch in 1024 2048 4096; do
    DAS_FILT_CHUNK=$ch timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s3/hub_ch$ch.json \
        2> gpurun_out/s3/hub_ch$ch.err || exit 14
done
for u in 8 16; do
    DAS_FILT_UNROLL=$u timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s3/hub_u$u.json \
        2> gpurun_out/s3/hub_u$u.err || exit 15
done
