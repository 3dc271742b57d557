set -o pipefail
mkdir -p gpurun_out/r6g
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread --durations=10 > gpurun_out/r6g/tests.txt 2>&1 || exit 1
timeout -k 10 300 python tools/fb_matched_profile.py 2>&1 | grep "ms\|median" > gpurun_out/r6g/fb.txt || exit 1
timeout -k 10 600 python bench.py --detail gpurun_out/r6g/bench_detail.json > gpurun_out/r6g/bench.json 2> gpurun_out/r6g/bench.err || exit 1
