#!/bin/bash
# time every build/ab/*/libbedgpu.so on the loader stage (GPU box); prints kernel avg per variant
cd $GRAFT_REPO_ROOT
for d in build/ab/*/; do
  n=$(basename $d)
  BEDGPU_LIB=$d/libbedgpu.so timeout -k 10 200 python3 bench.py --load-only --steps ${STEPS:-6} --warmup 1 --no-verify --no-cpu-baseline > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "$n FAILED"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));r=d['roofline'];print('%-12s %s avg %.4f ms  frac %.3f  step %.3f'%('$n',r['kernel'],r['avg_ms'],r['frac'],d['ms_per_step']))"
done
