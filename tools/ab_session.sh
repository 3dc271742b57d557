#!/bin/bash
# Scratch A/B session (run through gpurun): index-build parity, then bio join
# store variants and the build bench.  Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-materialise"
timeout -k 10 400 python -u -m pytest tests/test_gpu_index_build.py tests/test_gpu_golden.py tests/test_gpu_devgen.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_pidx.txt 2>&1 &&
timeout -k 10 300 python bench.py --workload build --no-cpu-baseline > gpurun_out/build_packed.json 2> gpurun_out/build.err &&
timeout -k 10 200 $B > gpurun_out/ab_plain.json 2> gpurun_out/ab.err &&
DAS_DJ_NT=1 timeout -k 10 200 $B > gpurun_out/ab_nt.json 2>> gpurun_out/ab.err &&
timeout -k 10 200 $B > gpurun_out/ab_plain2.json 2>> gpurun_out/ab.err &&
DAS_DJ_NT=1 timeout -k 10 200 $B > gpurun_out/ab_nt2.json 2>> gpurun_out/ab.err
