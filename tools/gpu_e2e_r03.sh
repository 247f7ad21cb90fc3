#!/bin/bash
# e2e breakdown of the drop-in CLI on the 100M x 100M inputs (page cache -> output file):
# N runs with BEDGPU_STATS=1 marks (one file per run) under gpurun_out/e2e_r03/<tag>/.
# usage: tools/gpu_e2e_r03.sh <tag> [runs] [extra env assignments...]
set -o pipefail
TAG=${1:-base}; RUNS=${2:-5}; shift 2 2>/dev/null
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/e2e_r03/$TAG; mkdir -p "$O"
D=/tmp/e2e; mkdir -p $D
[ -f $D/A.bed ] || ./tools/build/bedgen 100000000 42 > $D/A.bed || exit 1
[ -f $D/B.bed ] || ./tools/build/bedgen 100000000 43 > $D/B.bed || exit 1
( time cat $D/A.bed $D/B.bed > /dev/null ) 2> "$O/cat.txt"
for k in $(seq 1 "$RUNS"); do
  ( time env BEDGPU_STATS=1 "$@" timeout -k 10 120 python3 tools/e2e_time.py $D/out.bed ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed ) 2> "$O/run_$k.txt" || exit 1
done
sha256sum $D/out.bed | cut -c1-16 > "$O/sha.txt"
grep -h real "$O"/run_*.txt > "$O/real.txt"
cat "$O/real.txt"
