#!/bin/bash
# Scratch A/B session (run through gpurun): bio bench with and without scan
# views, and join unit shapes with views (variant libraries via DAS_MI355X_LIB).
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-materialise"
run() { timeout -k 10 200 env $1 $B > gpurun_out/w_$2.json 2>> gpurun_out/w.err; }
run "DAS_SCAN_VIEWS=1" views_g2 && run "DAS_SCAN_VIEWS=0" copy_g2 &&
run "DAS_MI355X_LIB=das_amd/variants/lib_g4_u4.so" views_g4 && run "DAS_MI355X_LIB=das_amd/variants/lib_g1_u4.so" views_g1 &&
run "DAS_SCAN_VIEWS=1" views_g2b && run "DAS_SCAN_VIEWS=0" copy_g2b &&
run "DAS_MI355X_LIB=das_amd/variants/lib_g4_u4.so" views_g4b
