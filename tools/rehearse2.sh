# Two ranks sharing cuda:0 over gloo (bench.py's rehearsal of the N-GPU
# path): the bench line of each workload, with collectives_per_step.
#   WORKLOADS="flybase bio" bash tools/rehearse2.sh
set -e
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in ${WORKLOADS:-flybase bio}; do
  DAS_BENCH_SAME_DEVICE=1 DAS_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --workload $w --gpus 2 \
    --steps ${STEPS:-5} --warmup ${WARMUP:-2} --no-cpu-baseline --no-materialise \
    --detail gpurun_out/rehearse2_${w}_detail.json > gpurun_out/rehearse2_$w.json 2> gpurun_out/rehearse2_$w.err
  echo "$w $(tail -1 gpurun_out/rehearse2_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('collectives_per_step'))")"
done
