#!/bin/bash
# closest-features chunk length sweep (BEDGPU_CLOSEST_CQ rows per chunk), 10M x 1B; outputs under gpurun_out/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
for cq in ${CQS:-64 128}; do
  BEDGPU_CLOSEST_CQ=$cq timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cq_$cq -- python3 bench.py --workload closest --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/cq_$cq.json 2> gpurun_out/cq_$cq.err || exit 1
done
echo done
