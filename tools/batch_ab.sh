# FlyBase / bio step with the step's queries batched (das_plan_execute_many)
# and one by one, alternating on one box
set -e
W=${WORKLOADS:-flybase}
for w in $W; do
  for b in 1 0 1 0; do
    timeout -k 10 300 python bench.py --workload $w --batch $b --steps 20 --warmup 5 --no-cpu-baseline --no-materialise --detail gpurun_out/ab_${w}_$b.json > gpurun_out/ab_${w}_$b.out 2> gpurun_out/ab_${w}_$b.err
    echo "$w batch=$b"; tail -1 gpurun_out/ab_${w}_$b.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('latency'))"
  done
done
