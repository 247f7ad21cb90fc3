#!/bin/bash
# SQ counters of the loader kernels (instruction mix, waits, LDS conflicts); outputs under gpurun_out/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
make -j16 all > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
B="python3 bench.py --load-only --steps 1 --warmup 1 --no-verify --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_sq1 -- $B > gpurun_out/pmc_sq1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmc_sq2 -- $B > gpurun_out/pmc_sq2.log 2>&1 || exit 1
echo done
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_SENDMSG --output-format csv -d gpurun_out/pmc_sq3 -- $B > gpurun_out/pmc_sq3.log 2>&1
echo done3
