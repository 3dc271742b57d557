#!/bin/bash
# Round-3 FlyBase latency diagnostics (gpurun from the repo root): the native
# plan timeline (DAS_TRACE marks), the host split per query and a cProfile of
# fresh anchors.  Each step under its own time limit, chained.
set -o pipefail
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
O=gpurun_out/diag
DAS_TRACE=1 timeout -k 10 200 python tools/trace_plan.py --cprofile $O/fb_cprofile.txt > $O/fb_trace.out 2> $O/fb_trace.txt &&
timeout -k 10 200 python tools/host_split.py > $O/fb_host_split.json 2> $O/fb_host_split.err
