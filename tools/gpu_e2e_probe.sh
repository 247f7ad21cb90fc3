#!/bin/bash
# e2e breakdown of the CLI on the 100M x 100M inputs (page cache -> file); outputs under gpurun_out/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
D=/tmp/e2e; mkdir -p $D
./tools/build/bedgen 100000000 42 > $D/A.bed && ./tools/build/bedgen 100000000 43 > $D/B.bed
( time cat $D/A.bed $D/B.bed > /dev/null ) 2> gpurun_out/e2e_cat.txt
for k in 1 2; do
  ( time BEDGPU_STATS=1 timeout -k 10 120 ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed > $D/out.bed ) 2> gpurun_out/e2e_cli_$k.txt || exit 1
done
sha256sum $D/out.bed | cut -c1-16 >> gpurun_out/e2e_cli_2.txt
( time timeout -k 10 120 ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed > /dev/null ) 2> gpurun_out/e2e_cli_null.txt
rm -rf $D
