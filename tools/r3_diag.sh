#!/bin/bash
# Round-3 diagnostics (gpurun from the repo root): the build leg on its own
# and after the hub leg (allocation trace), and the hub filtered expansion's
# fused / two-pass forms.  Each step under its own time limit, chained.
set -o pipefail
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
O=gpurun_out/diag
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 240 python bench.py --workload build $NB > $O/build_alone.json 2> $O/build_alone.err &&
DAS_ALLOC_TRACE=1 timeout -k 10 300 python bench.py --workload all --legs hub,build --steps 3 --warmup 1 $NB \
    > $O/hub_build.json 2> $O/hub_build.err &&
DAS_FILT_FUSED=0 timeout -k 10 240 python bench.py --workload hub $NB > $O/hub_fused0.json 2> $O/hub_fused0.err &&
DAS_FILT_FUSED=1 timeout -k 10 240 python bench.py --workload hub $NB > $O/hub_fused1.json 2> $O/hub_fused1.err &&
[ -x tools/ubench/cart_bw ] && timeout -k 10 60 tools/ubench/cart_bw 272048 1000 > $O/cart_bw.txt 2>&1 &&
timeout -k 10 60 tools/ubench/cart_bw 1000 272048 >> $O/cart_bw.txt 2>&1 &&
timeout -k 10 60 tools/ubench/cart_bw 20000000 14 >> $O/cart_bw.txt 2>&1
