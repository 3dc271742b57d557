#!/bin/bash
# Round-3 rocprof profiles (tools/profile_bench.sh) of the workloads named in
# $WLS (default: bio hub), chained; then the hub chunk-size A/B if CHUNK_AB=1.
set -o pipefail
export TMPDIR=/tmp
for w in ${WLS:-bio hub}; do
    TAG=r3 WORKLOAD=$w bash tools/profile_bench.sh || exit 20
done
if [ "${CHUNK_AB:-0}" = 1 ]; then bash tools/r3_hub_chunk.sh || exit 21; fi
exit 0
