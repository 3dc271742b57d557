#!/bin/bash
# Profiles bench.py on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 kernel trace + stats (csv) of the default bench run
#   2. HBM traffic PMC passes, FETCH_SIZE and WRITE_SIZE in separate runs
#      (MI355X_MICROARCH.md "HBM": one TCC counter group per pass)
#   3. tools/pmc_traffic.py -> gpurun_out/pmc_traffic.json (per-kernel bytes per
#      launch, gfx950 FETCH_SIZE correction applied)
# Copy what is worth keeping into profiles/ afterwards.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
ARGS="--steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/kt -o run -- python bench.py $ARGS > gpurun_out/prof_kt.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f rocpd -d gpurun_out/prof/fetch -o run -- python bench.py $ARGS > gpurun_out/prof_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f rocpd -d gpurun_out/prof/write -o run -- python bench.py $ARGS > gpurun_out/prof_write.log 2>&1 &&
python tools/pmc_traffic.py gpurun_out/prof/fetch gpurun_out/prof/write ${STEPS:-10} > gpurun_out/pmc_traffic.json
