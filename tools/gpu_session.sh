#!/bin/bash
# One GPU session (run through gpurun from the repo root).  MODES picks the
# steps, in order (default "tests profile"):
#   tests    the GPU parity suite (TESTS selects files, K a -k expression; default all)
#   bench    the default bench.py run exactly as the driver runs it
#            (BENCH_ARGS adds flags) -> gpurun_out/$TAG/bench.json + detail
#   profile  tools/profile_bench.sh for each workload in WORKLOADS (rocprof
#            kernel trace + FETCH/WRITE PMC passes + roofline check)
#   pmc      tools/pmc_kernel.sh (SQ / TCC counters) for KERNEL in WORKLOAD
#   cmd      an arbitrary command CMD (A/B runs), under CMD_TIMEOUT
# Steps are chained with &&, each under its own time limit, so a failure
# ends the session.
set -o pipefail
T=${TAG:-s}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
run_tests() {
    timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} ${K:+-k "$K"} -m gpu -x -v --timeout 150 \
        --timeout-method thread --durations=15 > gpurun_out/$T/tests.txt 2>&1
}
run_bench() {
    timeout -k 10 ${BENCH_TIMEOUT:-420} python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} \
        --detail gpurun_out/$T/bench_detail.json ${BENCH_ARGS:-} > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
}
run_profiles() {
    for w in ${WORKLOADS:-bio}; do
        TAG=$T WORKLOAD=$w bash tools/profile_bench.sh || return 1
    done
}
run_pmc() {
    WORKLOAD=${WORKLOAD:-hub} KERNEL="${KERNEL:-k_dj_filt<2}" bash tools/pmc_kernel.sh &&
    mkdir -p gpurun_out/$T/pmc && mv gpurun_out/pmc_${WORKLOAD:-hub}_* gpurun_out/$T/pmc/
}
run_cmd() {
    timeout -k 10 ${CMD_TIMEOUT:-300} bash -c "$CMD" > gpurun_out/$T/cmd.txt 2>&1
}
for m in ${MODES:-tests profile}; do
    case $m in
        tests) run_tests || exit 1 ;;
        bench) run_bench || exit 1 ;;
        profile) run_profiles || exit 1 ;;
        pmc) run_pmc || exit 1 ;;
        cmd) run_cmd || exit 1 ;;
        *) echo "unknown mode $m"; exit 2 ;;
    esac
done
