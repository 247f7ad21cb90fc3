#!/bin/bash
# HIP API + kernel trace of one CLI run on the 100M x 100M inputs (where the e2e time goes)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=/tmp/e2e; mkdir -p $D
./tools/build/bedgen 100000000 42 > $D/A.bed && ./tools/build/bedgen 100000000 43 > $D/B.bed
BEDGPU_STATS=1 timeout -k 10 120 ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed > /dev/null 2> gpurun_out/e2e_warm.txt
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/e2e_trace -- ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed > /dev/null 2> gpurun_out/e2e_trace.err
rm -rf $D
