# bench.py --workload $W under each environment setting of $CFGS (space-
# separated; "base" = none), alternating twice on one box
set -e
W=${W:-flybase}
CFGS=${CFGS:-base}
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in $CFGS; do
    tag=$(echo "$cfg" | tr '=,' '__')
    if [ "$cfg" = "base" ]; then envs=""; else envs=$(echo "$cfg" | tr ',' ' '); fi
    env $envs timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-materialise --detail gpurun_out/env_${W}_${tag}_$rep.json > gpurun_out/env_${W}_${tag}_$rep.out 2> gpurun_out/env_${W}_${tag}_$rep.err
    echo "$W $cfg rep $rep: $(tail -1 gpurun_out/env_${W}_${tag}_$rep.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'matched', d.get('step_ms_matched'), 'q2', (d.get('and_join_q2') or {}).get('us'), 'cart', (d.get('roofline') or {}).get('avg_launch_us'))")"
  done
done
