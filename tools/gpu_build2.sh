# one GPU call: build-path parity subset, 1e9-link build bench + kernel trace + PMC traffic
# (timed launches only: TOPK=2 keeps each kernel's two largest launches), hub trace + PMC traffic
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
D=gpurun_out/prof_build
mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_devgen.py tests/test_gpu_parity.py -k "devgen or build or reference_atoms or synthetic_matches or hub_four or incoming or keyspace or loader or composite" > gpurun_out/gpu_tests_build.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload build > gpurun_out/b_build.json 2> gpurun_out/b_build.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $D/kt -o run -- python bench.py --workload build > $D/kt.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f rocpd -d $D/fetch -o run -- python bench.py --workload build > $D/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f rocpd -d $D/write -o run -- python bench.py --workload build > $D/write.log 2>&1 &&
TOPK=2 python tools/pmc_traffic.py $D/fetch $D/write > gpurun_out/pmc_traffic_build.json &&
timeout -k 10 400 python -u bench.py --workload hub --steps 5 --warmup 1 > gpurun_out/b_hub.json 2> gpurun_out/b_hub.err &&
WORKLOAD=hub STEPS=3 bash tools/profile_bench.sh
