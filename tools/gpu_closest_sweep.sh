#!/bin/bash
# closest-features on the 10M x 1B workload with chunk parameters CQ/CW (BEDGPU_CLOSEST_CQ/_CW)
cd $GRAFT_REPO_ROOT
CQ=${CQ:-32}
CW=${CW:-8}
BEDGPU_CLOSEST_CQ=$CQ BEDGPU_CLOSEST_CW=$CW timeout -k 10 300 python3 bench.py --workload closest --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cl_${CQ}_${CW}.json 2> gpurun_out/cl_${CQ}_${CW}.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/cl_${CQ}_${CW}.json'));k=d['kernels_first_step_ms'];print('${CQ} ${CW}', d['ms_per_step'], k.get('k_closest_chunks'), k.get('k_closest_check'), k.get('k_closest_fix'), d['parity'])"
