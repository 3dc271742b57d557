#!/bin/bash
# Hub filtered-expansion chunk size A/B (DAS_FILT_CHUNK 1024 / 2048 / 4096)
set -o pipefail
mkdir -p gpurun_out/s3
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
for ch in 1024 2048 4096; do
    DAS_FILT_CHUNK=$ch timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s3/hub_ch$ch.json \
        2> gpurun_out/s3/hub_ch$ch.err || exit 14
done
DAS_CHUNK_UNIT=0 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s3/hub_cu0.json \
    2> gpurun_out/s3/hub_cu0.err || exit 15
