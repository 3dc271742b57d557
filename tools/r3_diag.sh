#!/bin/bash
# Round-3 diagnostics (gpurun from the repo root): the build leg now and at
# the round-2 tree (_r2/, same box), with the allocation trace; the hub
# filtered expansion's fused / two-pass forms; the cartesian microbenchmark.
# Each step under its own time limit, chained.
set -o pipefail
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
O=gpurun_out/diag
NB="--no-cpu-baseline --no-materialise"
R=$PWD
DAS_ALLOC_TRACE=1 timeout -k 10 240 python bench.py --workload build $NB > $O/build_alone.json 2> $O/build_alone.err &&
(cd _r2 && timeout -k 10 240 python bench.py --workload build --no-cpu-baseline > $R/$O/build_r2.json 2> $R/$O/build_r2.err) &&
DAS_FILT_FUSED=0 timeout -k 10 240 python bench.py --workload hub $NB > $O/hub_fused0.json 2> $O/hub_fused0.err &&
DAS_FILT_FUSED=1 timeout -k 10 240 python bench.py --workload hub $NB > $O/hub_fused1.json 2> $O/hub_fused1.err &&
timeout -k 10 60 tools/ubench/cart_bw 272048 1000 > $O/cart_bw.txt 2>&1 &&
timeout -k 10 60 tools/ubench/cart_bw 1000 272048 >> $O/cart_bw.txt 2>&1 &&
timeout -k 10 60 tools/ubench/cart_bw 20000000 14 >> $O/cart_bw.txt 2>&1
