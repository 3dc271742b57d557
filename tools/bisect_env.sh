set -o pipefail
mkdir -p gpurun_out/s3
T=tests/test_gpu_fullsize.py::test_gpu_bio_fullsize_counts
for cfg in "DAS_OWNER_SEARCH=1" "DAS_DIGEST_PREFIX=0" "DAS_L2I_PART=0" "DAS_DIGEST_PREFIX=0 DAS_L2I_PART=0 DAS_OWNER_SEARCH=1"; do
  echo "== $cfg" >> gpurun_out/s3/bisect.txt
  env $cfg timeout -k 10 150 python -u -m pytest $T -x -q --timeout 140 --timeout-method thread >> gpurun_out/s3/bisect.txt 2>&1
  rc=$?
  echo "rc=$rc" >> gpurun_out/s3/bisect.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
