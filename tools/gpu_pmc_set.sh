#!/bin/bash
# SQ counters of the headline step's kernels (instruction mix, issue, LDS) in two passes;
# outputs gpurun_out/pmc_set_sq{1,2}/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
B="python3 bench.py --steps 1 --warmup 1 --no-verify --no-cpu-baseline --no-e2e"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_set_sq1 -- $B > gpurun_out/pmc_set_sq1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmc_set_sq2 -- $B > gpurun_out/pmc_set_sq2.log 2>&1 || exit 1
echo done
