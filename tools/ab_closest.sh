#!/bin/bash
# closest-features A/B: every build/ab/*/libbedgpu.so at chunk sizes CQ in ${CQS:-32 16} (CW 8)
cd $GRAFT_REPO_ROOT
for d in build/ab/*/; do
  n=$(basename $d)
  for cq in ${CQS:-32 16}; do
    BEDGPU_LIB=$d/libbedgpu.so BEDGPU_CLOSEST_CQ=$cq BEDGPU_CLOSEST_CW=8 timeout -k 10 200 python3 bench.py --workload closest --steps 2 --warmup 1 --no-cpu-baseline --no-verify > gpurun_out/abc_${n}_$cq.json 2> gpurun_out/abc_${n}_$cq.err || { echo "$n $cq FAILED"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abc_${n}_$cq.json'));k=d['kernels_first_step_ms'];print('%-10s %3s step %.1f chunks %.2f check %s fix %s'%('$n','$cq',d['ms_per_step'],k.get('k_closest_chunks'),k.get('k_closest_check'),k.get('k_closest_fix')))"
  done
done
