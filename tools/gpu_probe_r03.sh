#!/bin/bash
# round-3 e2e probe: ingest micro-benchmarks (tools/e2e_probe.cpp) and a runtime/kernel trace
# of the drop-in CLI on 100M x 100M, outputs under gpurun_out/probe_r03/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/probe_r03; mkdir -p "$O"
D=/tmp/e2e; mkdir -p $D
[ -f $D/A.bed ] || ./tools/build/bedgen 100000000 42 > $D/A.bed || exit 1
[ -f $D/B.bed ] || ./tools/build/bedgen 100000000 43 > $D/B.bed || exit 1
df -h /tmp > "$O/df.txt"; mount | grep -E ' /tmp | / ' >> "$O/df.txt"
true
for k in 1 2 3; do ( time env BEDGPU_STATS=1 timeout -k 10 120 ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed > $D/out.bed ) 2> "$O/cli_$k.txt" || exit 1; done
cd /tmp
BEDGPU_FULL_EXIT=1 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --stats --output-format csv \
  -d "$GRAFT_REPO_ROOT/$O/trace" -o cli -- "$GRAFT_REPO_ROOT/bedops_amd/bin/bedops" --intersect $D/A.bed $D/B.bed > $D/out.bed || exit 1
cd "$GRAFT_REPO_ROOT"
sha256sum $D/out.bed | cut -c1-16 > "$O/sha.txt"
grep -h real "$O"/cli_*.txt
