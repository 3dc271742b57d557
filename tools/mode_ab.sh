# bench.py --workload $W with --batch 1 and --batch 0 alternating (REPS
# pairs) on one box; each run also times the other mode on fresh anchors, so
# every pair gives both modes in both orders.  ENVS: env settings for all runs;
# MODES (default "1 0"): the --batch values, a ":none" suffix adding
# --events none (no HIP events in the timed steps: the events' own cost).
set -e
W=${W:-bio}
for rep in $(seq 1 ${REPS:-2}); do
  for m in ${MODES:-1 0}; do
    b=${m%%:*}
    extra=""
    case $m in *:none) extra="--events none" ;; esac
    out=gpurun_out/mode_${W}_b$(echo $m | tr ':' '_')_$rep
    env $ENVS timeout -k 10 300 python bench.py --workload $W --batch $b --steps 20 --warmup 5 --no-cpu-baseline \
        --no-materialise $extra --detail $out.json > $out.out 2> $out.err
    echo "$W mode=$m rep $rep: $(tail -1 $out.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('timed', d['ms_per_step'], 'batched', d.get('step_ms_batched'), 'matched', d.get('step_ms_matched'), 'box', (d.get('box') or {}).get('store16_nt_GBps'))")"
  done
done
