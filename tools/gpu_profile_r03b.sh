#!/bin/bash
# Round-3 profiling recipe (GPU box): per workload a kernel trace + stats run, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes reduced to per-launch HBM bytes
# (tools/pmc_traffic.py -> gpurun_out/pmc_traffic_<workload>.json); then the headline bench
# line (CPU baselines + file->file CLI). Outputs under gpurun_out/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
T=${TAG:-r03b}
for w in ${WORKLOADS:-intersect}; do
  B="python3 bench.py --workload $w --no-cpu-baseline --no-e2e"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_${w}_trace -- $B --steps 5 --warmup 1 > gpurun_out/${T}_${w}_trace.json 2> gpurun_out/${T}_${w}_trace.err || exit 1
  if [ -z "$NO_PMC" ]; then
    timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_${w}_fetch -- $B --steps 1 --warmup 1 --no-verify > gpurun_out/${T}_${w}_fetch.json 2> gpurun_out/${T}_${w}_fetch.err || exit 1
    timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_${w}_write -- $B --steps 1 --warmup 1 --no-verify > gpurun_out/${T}_${w}_write.json 2> gpurun_out/${T}_${w}_write.err || exit 1
    python3 tools/pmc_traffic.py gpurun_out/${T}_${w}_fetch gpurun_out/${T}_${w}_write gpurun_out/pmc_traffic_${w}.json || exit 1
  fi
  echo "$w profiled"
done
[ -n "$NO_BENCH" ] || timeout -k 10 700 python3 bench.py --steps 10 --warmup 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
cat gpurun_out/${T}_bench.json
echo ALLDONE
