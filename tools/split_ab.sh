#!/bin/bash
# The bio (or $W) step under rocprofv3 kernel traces, one run per setting of
# $CFGS (space-separated; "base" = the default batch; "b0" / "b1" = --batch 0 / 1; other
# entries are comma-separated env settings), in the order given, then
# tools/step_split.py over each trace -> gpurun_out/split_<W>_<SES>/<cfg>_<k>/split.json.
# Every GPU step has its own time limit; a failure ends the script.
set -o pipefail
W=${W:-bio}
CFGS=${CFGS:-"base b0 base b0"}
export TMPDIR=/tmp
k=0
for cfg in $CFGS; do
  k=$((k + 1))
  tag=$(echo "$cfg" | tr '=,' '__')_$k
  args="--workload $W --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-cpu-baseline --no-materialise --no-extras"
  envs=""
  if [ "$cfg" = "b0" ] || [ "$cfg" = "b1" ]; then args="$args --batch ${cfg#b}"; elif [ "$cfg" != "base" ]; then envs=$(echo "$cfg" | tr ',' ' '); fi
  D=gpurun_out/split_${W}_${SES:-s}/$tag
  mkdir -p $D
  env $envs timeout -k 10 ${PROF_TIMEOUT:-240} rocprofv3 --kernel-trace -f csv -d $D -o run -- python bench.py $args \
      --detail $D/detail.json > $D/bench.out 2> $D/bench.err || exit 1
  python tools/step_split.py "$(find $D -name 'run_kernel_trace.csv' | head -n 1)" ${STEPS:-20} "$W $cfg" \
      > $D/split.json || exit 1
  echo "$W $cfg: $(tail -1 $D/bench.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], 'cart', (d.get('roofline') or {}).get('avg_launch_us'), 'store', (d.get('box') or {}).get('store16_nt_GBps'))") $(python -c "import json; r=json.load(open('$D/split.json'))['regions'][0]; print('wall', r['wall_us'], 'busy', r['busy_us'], 'idle', r['idle_us'], 'overlap', r['overlap_us'])")"
  find $D -name '*.csv' ! -name 'run_kernel_trace.csv' -delete
done
