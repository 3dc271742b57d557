#!/bin/bash
# SQ counter passes over the join microbenchmark (one rocprofv3 --pmc run per pass).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc/p1 -o run -- python tools/ubench_join.py --reps 2 > gpurun_out/pmc_p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d gpurun_out/pmc/p2 -o run -- python tools/ubench_join.py --reps 2 > gpurun_out/pmc_p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d gpurun_out/pmc/p3 -o run -- python tools/ubench_join.py --reps 2 > gpurun_out/pmc_p3.log 2>&1
