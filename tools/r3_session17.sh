#!/bin/bash
# Round 3, session 17: the opt-in join build (DAS_DJ_BUILD=sparse) and the
# small compaction carrying the semi-join guard (DAS_SMALL_GUARD=1) under the
# golden / hub / semi-join GPU tests, then the bio step with and without them.
set -o pipefail
mkdir -p gpurun_out/s17
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise --no-extras"
DAS_DJ_BUILD=sparse DAS_SMALL_GUARD=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py \
    -m gpu -x -q --timeout 200 --timeout-method thread -k "synthetic or hub_join or semi_join or hub_four" \
    > gpurun_out/s17/tests_optin.txt 2>&1 &&
timeout -k 10 100 python bench.py --workload bio $NB > gpurun_out/s17/bio_default.json 2> gpurun_out/s17/bio_default.err &&
DAS_DJ_BUILD=sparse DAS_SMALL_GUARD=1 timeout -k 10 100 python bench.py --workload bio $NB > gpurun_out/s17/bio_optin.json 2> gpurun_out/s17/bio_optin.err
