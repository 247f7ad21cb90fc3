#!/bin/bash
# HIP initialisation on the box: agents HSA sees, bare init under visibility settings, and
# the CLI's e2e with them; gpurun_out/init_r03/summary.txt
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/init_r03; mkdir -p $O
( timeout -k 5 60 rocminfo | grep -E "Marketing Name|Name: +gfx" ) > $O/rocminfo.txt 2>&1
ls /dev/dri >> $O/rocminfo.txt 2>&1
P=./tools/build/exit_probe
: > $O/summary.txt
for V in "plain:" "rocr0:ROCR_VISIBLE_DEVICES=0" "hip0:HIP_VISIBLE_DEVICES=0"; do
  lab=${V%%:*}; envs=${V#*:}
  for k in 1 2 3 4 5; do
    out=$(env $envs timeout -k 5 60 $P streams 0) || { echo "$lab failed" >> $O/summary.txt; exit 1; }
    echo "$lab $k: $(echo "$out" | grep setdevice)" >> $O/summary.txt
  done
done
D=/tmp/e2e; mkdir -p $D
[ -f $D/A.bed ] || ./tools/build/bedgen 100000000 42 > $D/A.bed || exit 1
[ -f $D/B.bed ] || ./tools/build/bedgen 100000000 43 > $D/B.bed || exit 1
cat $D/A.bed $D/B.bed > /dev/null
for V in "plain:" "rocr0:ROCR_VISIBLE_DEVICES=0"; do
  lab=${V%%:*}; envs=${V#*:}
  for k in 1 2 3 4; do
    env $envs BEDGPU_STATS=1 timeout -k 10 120 python3 tools/e2e_time.py $D/out.bed ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed 2> "$O/${lab}_$k.txt" || exit 1
    echo "$lab $k: $(grep -h '^split' "$O/${lab}_$k.txt") | $(grep -h 'bedgpu host' "$O/${lab}_$k.txt" | awk '{printf "%s%s ", $3, $NF}')" >> "$O/summary.txt"
  done
done
cat $O/rocminfo.txt $O/summary.txt
