set -e
for g in auto 0 auto 0; do
  if [ "$g" = "auto" ]; then unset DAS_CHAIN_GRID; else export DAS_CHAIN_GRID=$g; fi
  timeout -k 10 300 python bench.py --workload flybase --steps 20 --warmup 5 --no-cpu-baseline --no-materialise --detail gpurun_out/fb_$g.json > gpurun_out/fb_$g.out 2> gpurun_out/fb_$g.err
  echo "grid=$g"; tail -1 gpurun_out/fb_$g.out | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('latency'))"
done
