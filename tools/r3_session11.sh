#!/bin/bash
# Direct-address join range floor 2^22 (small joins over wide key ranges sort
# instead): parity tests of the join paths, bio A/B against the round-3 floor
# 2^26, bio plan trace.
set -o pipefail
mkdir -p gpurun_out/s12
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "golden or join or reference or bio or template" > gpurun_out/s12/tests1.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload bio $NB > gpurun_out/s12/bio.json 2> gpurun_out/s12/bio.err &&
DAS_DJ_RANGE_FLOOR=26 timeout -k 10 200 python bench.py --workload bio $NB > gpurun_out/s12/bio_f26.json 2> gpurun_out/s12/bio_f26.err &&
DAS_TRACE=1 timeout -k 10 200 python tools/trace_plan.py --workload bio > gpurun_out/s12/bio_trace.out 2> gpurun_out/s12/bio_trace.txt
