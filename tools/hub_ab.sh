# A/B of an env knob on the hub leg (config 5), alternating, one box:
#   KNOB=DAS_FILT_RUN bash tools/hub_ab.sh
set -e
for v in ${VALUES:-1 0 1 0}; do
  export $KNOB=$v
  timeout -k 10 300 python bench.py --workload hub --steps 20 --warmup 5 --no-cpu-baseline --no-materialise \
    --detail gpurun_out/hub_ab_$v.json > gpurun_out/hub_ab_$v.out 2> gpurun_out/hub_ab_$v.err
  echo "$KNOB=$v $(tail -1 gpurun_out/hub_ab_$v.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['ms_per_step'], r['kernel'], r['frac'], r['avg_launch_us'])")"
done
