#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
make -j16 all > gpurun_out/build.log 2>&1 || exit 1
for st in 1 2 0; do
  BEDGPU_PARSE_STOP=$st timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_stop$st -- python3 bench.py --load-only --steps 1 --warmup 1 --no-verify --no-cpu-baseline > gpurun_out/pmc_stop$st.log 2>&1 || exit 1
  BEDGPU_PARSE_STOP=$st timeout -k 10 200 python3 bench.py --load-only --steps 10 --warmup 2 --no-verify --no-cpu-baseline > gpurun_out/time_stop$st.json 2>/dev/null || exit 1
done
echo done
