#!/bin/bash
# Profiles bench.py on the GPU box (run through gpurun from the repo root):
# host cProfile, rocprofv3 kernel trace + stats, and the HBM traffic PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate runs, MI355X_MICROARCH.md "HBM").
# Outputs land under gpurun_out/; the summaries worth keeping are copied into
# profiles/ by hand.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
ARGS="--steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 300 python -u bench.py $ARGS --cprofile gpurun_out/cprof.txt > gpurun_out/bench_cprof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o run -- python bench.py $ARGS > gpurun_out/prof_kt.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_write.log 2>&1
