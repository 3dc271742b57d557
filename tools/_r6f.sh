set -o pipefail
mkdir -p gpurun_out/r6f
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -m gpu -x -v --timeout 150 --timeout-method thread -k "chain or fused or flybase or plan_execute_many or golden" > gpurun_out/r6f/tests.txt 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 300 python tools/fb_matched_profile.py 2>&1 | grep "ms\|median" > gpurun_out/r6f/fb_noprep_$r.txt || exit 1
DAS_CHAIN_PREP1=1 timeout -k 10 300 python tools/fb_matched_profile.py 2>&1 | grep "ms\|median" > gpurun_out/r6f/fb_prep_$r.txt || exit 1
done
