#!/bin/bash
# One-walk filtered expansion as the default, key directories up to 16 id
# slots per key, bucket directories elsewhere, the one walk in MALL-sized
# pieces (A/B): parity tests, hub / FlyBase / build legs, bio plan trace.
set -o pipefail
mkdir -p gpurun_out/s11
export TMPDIR=/tmp
NB="--no-cpu-baseline --no-materialise"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    -k "semi_join_multi or hub or index_join or flybase or golden or chain or anti" > gpurun_out/s11/tests1.txt 2>&1 &&
timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s11/hub.json 2> gpurun_out/s11/hub.err &&
DAS_FILT_PIECE_KB=65536 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s11/hub_p64.json 2> gpurun_out/s11/hub_p64.err &&
DAS_FILT_PIECE_KB=131072 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s11/hub_p128.json 2> gpurun_out/s11/hub_p128.err &&
DAS_KEY_DIR_SPARSE=0 DAS_KEY_BDIR=0 timeout -k 10 200 python bench.py --workload hub $NB > gpurun_out/s11/hub_dense.json 2> gpurun_out/s11/hub_dense.err &&
timeout -k 10 200 python bench.py --workload flybase --steps 20 --warmup 3 $NB > gpurun_out/s11/fb.json 2> gpurun_out/s11/fb.err &&
DAS_KEY_DIR_SPARSE=0 DAS_KEY_BDIR=0 timeout -k 10 200 python bench.py --workload flybase --steps 20 --warmup 3 $NB > gpurun_out/s11/fb_dense.json 2> gpurun_out/s11/fb_dense.err &&
timeout -k 10 300 python bench.py --workload build $NB > gpurun_out/s11/build.json 2> gpurun_out/s11/build.err &&
DAS_KEY_DIR_SPARSE=0 DAS_KEY_BDIR=0 timeout -k 10 300 python bench.py --workload build $NB > gpurun_out/s11/build_dense.json 2> gpurun_out/s11/build_dense.err &&
DAS_TRACE=1 timeout -k 10 200 python tools/trace_plan.py --workload bio > gpurun_out/s11/bio_trace.out 2> gpurun_out/s11/bio_trace.txt
