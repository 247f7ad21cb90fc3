#!/bin/bash
# e2e CLI (page cache -> output file) on the 100M x 100M inputs, per reader-ring setting
# (BEDGPU_RD_THREADS x BEDGPU_RD_CHUNK_MB [x BEDGPU_RD_STREAMS]), with the host phase marks (BEDGPU_STATS=1).
# Outputs gpurun_out/e2e_sweep_<threads>x<chunk>.txt; every run's output hash is checked.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
D=/tmp/e2e; mkdir -p $D
./tools/build/bedgen 100000000 42 > $D/A.bed && ./tools/build/bedgen 100000000 43 > $D/B.bed || exit 1
cat $D/A.bed $D/B.bed > /dev/null
timeout -k 10 120 ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed > $D/out.bed || exit 1  # warm
for cfg in ${CFGS:-8x16 16x16 16x8 24x8 32x4}; do
  IFS=x read -r t m st <<< "$cfg"
  f=gpurun_out/e2e_sweep_$cfg.txt
  for k in 1 2 3; do
    ( time BEDGPU_STATS=1 BEDGPU_RD_THREADS=$t BEDGPU_RD_CHUNK_MB=$m BEDGPU_RD_STREAMS=${st:-2} timeout -k 10 120 \
        ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed > $D/out.bed ) 2>> $f || exit 1
  done
  sha256sum $D/out.bed | cut -c1-16 >> $f
  echo "$cfg done"
done
rm -rf $D
