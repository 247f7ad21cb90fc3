#!/bin/bash
# Bench lines for every BASELINE.json config on the GPU path (outputs under gpurun_out/).
cd $GRAFT_REPO_ROOT
make -j16 all > gpurun_out/build.log 2>&1 || exit 1
for w in intersect element-of bedmap closest; do
  timeout -k 10 500 python3 bench.py --workload $w --steps ${STEPS:-5} --warmup 1 > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err || exit 1
  echo "$w: $(cut -c1-200 gpurun_out/wl_$w.json)"
done
