#!/bin/bash
# SQ instruction counters of one bench step (intersect): per-kernel VALU / SALU / LDS / VMEM
# instruction counts and wait cycles, two rocprofv3 --pmc passes (<= 8 SQ counters each)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${ROUND:-r05}_${TAG:-sq}
mkdir -p $O
W=${WORKLOAD:-intersect}
timeout -s KILL ${PMC_T:-120} rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH \
  --output-format csv -d $O/sq1 -- python3 bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-verify \
  > $O/sq1.json 2> $O/sq1.err || { tail -5 $O/sq1.err; exit 1; }
timeout -s KILL ${PMC_T:-120} rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS \
  --output-format csv -d $O/sq2 -- python3 bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-verify \
  > $O/sq2.json 2> $O/sq2.err || { tail -5 $O/sq2.err; exit 1; }
if [ -n "$SQ3" ]; then  # optional third pass (counter names vary by ROCm release)
  timeout -s KILL 60 rocprofv3 --pmc $SQ3 \
    --output-format csv -d $O/sq3 -- python3 bench.py --workload $W --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-verify \
    > $O/sq3.json 2> $O/sq3.err || tail -5 $O/sq3.err
fi
python3 tools/sq_summary.py $O/sq1 $O/sq2 $( [ -d $O/sq3 ] && echo $O/sq3 ) --kernel ${KSUB:-k_parse_set} > $O/sq_summary.txt || exit 1
cat $O/sq_summary.txt
echo SQDONE
