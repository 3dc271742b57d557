#!/bin/bash
# rocprof profiles of the FlyBase and build legs, then the FlyBase host split.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s8
WLS="flybase build" CHUNK_AB=0 bash tools/r3_profiles.sh &&
timeout -k 10 200 python tools/host_split.py > gpurun_out/s8/fb_host_split.json 2> gpurun_out/s8/fb_host_split.err
