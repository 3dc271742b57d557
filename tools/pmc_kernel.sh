#!/bin/bash
# SQ / TCC counter passes (one rocprofv3 --pmc run per pass) over a short
# bench.py run; tools/pmc_summary.py then prints the counters of the last
# dispatches of one kernel:  KERNEL='k_dj_write<2, 1' WORKLOAD=bio bash tools/pmc_kernel.sh
set -o pipefail
W=${WORKLOAD:-bio}
D=/tmp/pmc_$W    # databases stay on the box (gpurun_out is merged back only below 64 MiB)
mkdir -p $D
export TMPDIR=/tmp
ARGS="--workload $W --steps 3 --warmup 2 --no-cpu-baseline --no-materialise ${BENCH_ARGS:-}"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $D/p1 -o run -- python bench.py $ARGS > gpurun_out/pmc_${W}_p1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $D/p2 -o run -- python bench.py $ARGS > gpurun_out/pmc_${W}_p2.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $D/p3 -o run -- python bench.py $ARGS > gpurun_out/pmc_${W}_p3.log 2>&1 &&
python tools/pmc_summary.py "${KERNEL:-k_dj_write<2, 1}" $(find $D -name '*.db') > gpurun_out/pmc_${W}_summary.txt
