#!/bin/bash
# GPU-box profiling recipe: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes, then a full bench line (with cpu_baseline). Outputs under gpurun_out/.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
make -j16 all > gpurun_out/build.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG:-r01v6}_trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG:-r01v6}_trace.json 2> gpurun_out/prof_${TAG:-r01v6}_trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${TAG:-r01v6}_fetch -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify > gpurun_out/prof_${TAG:-r01v6}_fetch.json 2> gpurun_out/prof_${TAG:-r01v6}_fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_${TAG:-r01v6}_write -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify > gpurun_out/prof_${TAG:-r01v6}_write.json 2> gpurun_out/prof_${TAG:-r01v6}_write.err
timeout -k 10 500 python3 bench.py --steps 10 --warmup 2 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
echo ALLDONE
