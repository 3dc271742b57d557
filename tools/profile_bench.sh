#!/bin/bash
# Measures one bench.py workload on the GPU box (run through gpurun from the
# repo root); every step has its own time limit and the steps are chained, so
# a failure ends the script.
#   1. bench.py itself (the JSON line, with its cpu_baseline)
#   2. rocprofv3 kernel trace + stats (csv) of the same bench command
#   3. HBM traffic PMC passes, FETCH_SIZE and WRITE_SIZE in separate runs
#      (MI355X_MICROARCH.md "HBM": one TCC counter group per pass)
#   4. tools/pmc_traffic.py -> per-kernel bytes per launch (gfx950 FETCH_SIZE
#      correction), tools/roofline_check.py -> the roofline of the bench line
#      printed UNDER rocprof recomputed from the rocprof trace of the same
#      process's timed launches (those between bench.py's k_prof_mark brackets)
# WORKLOAD selects bench.py --workload (default bio); BENCH_ARGS adds flags;
# TAG names the outputs gpurun_out/<TAG>_<workload>*, and <TAG>_<workload>_box.txt
# records the card (serial, unique id, clocks).  Copy what is worth keeping
# into profiles/ afterwards.
set -o pipefail
W=${WORKLOAD:-bio}
T=${TAG:-r2}
D=gpurun_out/prof_${T}_$W
mkdir -p $D
export TMPDIR=/tmp
ARGS="--workload $W --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${BENCH_ARGS:-}"
# which box: the card's serial / unique id and its clocks next to the records
# (box-to-box spreads of the write-bound kernels are then attributable)
{ date -u; hostname; rocm-smi --showserial --showuniqueid --showclocks 2>&1 || true; } > gpurun_out/${T}_${W}_box.txt
PARGS="$ARGS --no-cpu-baseline --no-materialise --no-extras"
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $ARGS --detail gpurun_out/${T}_bench_${W}_detail.json > gpurun_out/${T}_bench_$W.json 2> $D/bench.err &&
timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -f csv -d $D/kt -o run -- python bench.py $PARGS --detail $D/kt_detail.json > $D/kt.log 2>&1 &&
cp "$(find $D/kt -name 'run_kernel_stats.csv' | head -n 1)" gpurun_out/${T}_${W}_kernel_stats.csv &&
cp "$(find $D/kt -name 'run_kernel_trace.csv' | head -n 1)" gpurun_out/${T}_${W}_kernel_trace.csv &&
timeout -s KILL ${PROF_TIMEOUT:-300} rocprofv3 --pmc FETCH_SIZE -f rocpd -d $D/fetch -o run -- python bench.py $PARGS --detail $D/fetch_detail.json > $D/fetch.log 2>&1 &&
timeout -s KILL ${PROF_TIMEOUT:-300} rocprofv3 --pmc WRITE_SIZE -f rocpd -d $D/write -o run -- python bench.py $PARGS --detail $D/write_detail.json > $D/write.log 2>&1 &&
if [ "$W" = build ]; then export LAST_FROM=gpurun_out/${T}_bench_$W.json; fi &&
python tools/pmc_traffic.py $D/fetch $D/write > gpurun_out/${T}_pmc_traffic_$W.json &&
cp $D/kt.log gpurun_out/${T}_bench_${W}_under_rocprof.log &&
python tools/roofline_check.py $D/kt.log gpurun_out/${T}_${W}_kernel_stats.csv \
    gpurun_out/${T}_pmc_traffic_$W.json gpurun_out/${T}_${W}_kernel_trace.csv > gpurun_out/${T}_roofline_check_$W.json
