#!/bin/bash
# Round-3 GPU session (run through gpurun from the repo root): the selected
# GPU tests (TESTK = pytest -k expression, default all), the default bench
# run (every workload), and a 2-rank rehearsal of the N-GPU bench path on one
# GPU over gloo at reduced sizes.  Steps are chained with &&, each under its
# own time limit, so a failure ends the session.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${TESTK:-}
run_tests() {
    if [ -n "$K" ]; then
        timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -x -v --timeout 300 \
            --timeout-method thread -k "$K" > gpurun_out/r3_tests.txt 2>&1
    else
        timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -x -v --timeout 300 \
            --timeout-method thread --durations=15 > gpurun_out/r3_tests.txt 2>&1
    fi
}
run_bench() {
    timeout -k 10 ${BENCH_TIMEOUT:-500} python bench.py --steps 10 --warmup 3 \
        > gpurun_out/r3_bench_all.json 2> gpurun_out/r3_bench_all.err
}
run_rehearsal() {
    DAS_BENCH_SAME_DEVICE=1 DAS_DIST_BACKEND=gloo timeout -k 10 ${REH_TIMEOUT:-500} \
        python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
        bench.py --steps 3 --warmup 1 --legs flybase,hub,build --genes 20000 --members 2000000 --bps 5000 \
        --inheritance 10000 --fb-genes 30000 --fb-rows 45000 --hub-links 20000000 --hub-nodes 1000000 \
        --links 20000000 --nodes 1000000 --no-cpu-baseline > gpurun_out/r3_rehearse2.json 2> gpurun_out/r3_rehearse2.err
}
for s in $(echo "${STEPS:-tests,bench,rehearsal}" | tr , ' '); do
    case $s in
        tests) run_tests || exit 11 ;;
        bench) run_bench || exit 12 ;;
        rehearsal) run_rehearsal || exit 13 ;;
    esac
done
exit 0
