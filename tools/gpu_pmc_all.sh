#!/bin/bash
# SQ counters of every kernel of one bench step (instruction mix, waits, LDS conflicts); outputs under gpurun_out/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
W=${WORKLOAD:-intersect}
B="python3 bench.py --workload $W --steps 1 --warmup 1 --no-verify --no-cpu-baseline --no-e2e"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcall_${W}_sq1 -- $B > gpurun_out/pmcall_${W}_sq1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmcall_${W}_sq2 -- $B > gpurun_out/pmcall_${W}_sq2.log 2>&1 || exit 1
echo done
