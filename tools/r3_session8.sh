#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/s9
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "union or flybase or golden or shape" > gpurun_out/s9/tests.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload flybase --steps 20 --warmup 3 $NB > gpurun_out/s9/fb.json 2> gpurun_out/s9/fb.err &&
timeout -k 10 200 python tools/host_split.py > gpurun_out/s9/fb_host_split.json 2> gpurun_out/s9/fb_host_split.err
