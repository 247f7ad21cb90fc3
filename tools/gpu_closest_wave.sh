#!/bin/bash
# closest-features, one wave per chunk: parity first, then the 10M x 1B bench per chunk length
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "closest" > gpurun_out/cw_tests.log 2>&1 || { echo tests failed; exit 1; }
for cq in ${CQS:-32 64 128}; do
  BEDGPU_CLOSEST_CQ=$cq timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cw_$cq -- python3 bench.py --workload closest --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/cw_$cq.json 2> gpurun_out/cw_$cq.err || exit 1
done
echo done
