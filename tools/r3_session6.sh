#!/bin/bash
# Filtered-expansion tests (incl. the one-launch MODE 2), hub one-pass A/B,
# then rocprof profiles ($WLS, default bio hub).  Chained.
set -o pipefail
mkdir -p gpurun_out/s7 gpurun_out/s3
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "semi_join or hub" > gpurun_out/s7/tests.txt 2>&1 &&
DAS_FILT_ONEPASS=1 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s3/hub_onepass.json \
    2> gpurun_out/s3/hub_onepass.err &&
timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s3/hub_twopass.json 2> gpurun_out/s3/hub_twopass.err &&
WLS="${WLS:-bio hub}" CHUNK_AB=0 bash tools/r3_profiles.sh
