set -o pipefail
mkdir -p gpurun_out/r6e
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 150 --timeout-method thread -k "semi_join_multi or hub" > gpurun_out/r6e/tests.txt 2>&1 || exit 1
W=hub CFGS="base DAS_FILT_STAGED=0 DAS_FILT_CUNIT=0" timeout -k 10 400 bash tools/env_ab.sh > gpurun_out/r6e/hub_ab.txt 2>&1 || exit 1
python - <<'PY' >> gpurun_out/r6e/hub_ab.txt
import json, glob
for f in sorted(glob.glob("gpurun_out/env_hub_*.json")):
    d = json.load(open(f)); k = d.get("kernels", {})
    print(f, {n: v["avg_us"] for n, v in list(k.items())[:6]})
PY
timeout -k 10 300 python tools/fb_matched_profile.py > gpurun_out/r6e/fb_prof.txt 2>&1 || exit 1
DAS_TRACE=1 timeout -k 10 300 python tools/fb_matched_profile.py > /dev/null 2> gpurun_out/r6e/fb_trace.txt || exit 1
