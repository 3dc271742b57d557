#!/bin/bash
# A/B of one environment switch on one bench.py workload, alternating runs
# (A B A B) in fresh processes on one box:
#   AB_VAR=DAS_OWNER_SEARCH AB_A=0 AB_B=1 WORKLOAD=hub TAG=s3 bash tools/ab.sh
# Lines go to gpurun_out/$TAG/ab_<workload>_<var>.jsonl (one compact bench
# line per run, prefixed with the setting).
set -o pipefail
T=${TAG:-ab}
W=${WORKLOAD:-bio}
mkdir -p gpurun_out/$T
OUT=gpurun_out/$T/ab_${W}_${AB_VAR}.jsonl
: > $OUT
for v in ${AB_A} ${AB_B} ${AB_A} ${AB_B}; do
    env $AB_VAR=$v timeout -k 10 ${AB_TIMEOUT:-240} python bench.py --workload $W --steps ${STEPS:-10} \
        --warmup ${WARMUP:-3} --no-cpu-baseline --no-materialise ${BENCH_ARGS:-} \
        --detail gpurun_out/$T/ab_${W}_${AB_VAR}_$v.json > gpurun_out/$T/ab_line.json \
        2> gpurun_out/$T/ab_${W}.err || exit 1
    echo "{\"$AB_VAR\": \"$v\", \"line\": $(tail -n 1 gpurun_out/$T/ab_line.json)}" >> $OUT
done
