#!/bin/bash
# Profiles bench.py on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 kernel trace + stats (csv) of the bench run
#   2. HBM traffic PMC passes, FETCH_SIZE and WRITE_SIZE in separate runs
#      (MI355X_MICROARCH.md "HBM": one TCC counter group per pass)
#   3. tools/pmc_traffic.py -> gpurun_out/pmc_traffic[_<workload>].json (per-kernel
#      bytes per launch, gfx950 FETCH_SIZE correction applied)
# WORKLOAD selects bench.py --workload (default bio); BENCH_ARGS adds flags.
# Copy what is worth keeping into profiles/ afterwards.
set -o pipefail
W=${WORKLOAD:-bio}
D=gpurun_out/prof_$W
mkdir -p $D
export TMPDIR=/tmp
ARGS="--workload $W --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-}"
OUT=pmc_traffic.json
[ "$W" != bio ] && OUT=pmc_traffic_$W.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/kt -o run -- python bench.py $ARGS > $D/kt.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f rocpd -d $D/fetch -o run -- python bench.py $ARGS > $D/fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f rocpd -d $D/write -o run -- python bench.py $ARGS > $D/write.log 2>&1 &&
python tools/pmc_traffic.py $D/fetch $D/write > gpurun_out/$OUT
