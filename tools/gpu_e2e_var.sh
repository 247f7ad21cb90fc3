#!/bin/bash
# e2e variants of the drop-in CLI on the 100M x 100M inputs (page cache -> output file):
# each VARIANT is "label:ENV=V,ENV=V" (empty env = default); 3 runs each with BEDGPU_STATS
# marks; summary in gpurun_out/e2e_var/<tag>/summary.txt. Also a bare HIP-init probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/e2e_var/${TAG:-v}; mkdir -p "$O"
D=/tmp/e2e; mkdir -p $D
[ -f $D/A.bed ] || ./tools/build/bedgen 100000000 42 > $D/A.bed || exit 1
[ -f $D/B.bed ] || ./tools/build/bedgen 100000000 43 > $D/B.bed || exit 1
cat $D/A.bed $D/B.bed > /dev/null
nproc > "$O/env.txt"; cat /sys/fs/cgroup/cpu.max >> "$O/env.txt" 2>/dev/null; free -g >> "$O/env.txt"
if [ -x tools/build/exit_probe ]; then
  for k in 1 2 3; do
    s=$(python3 -c 'import time;print("%.6f"%time.monotonic())')
    timeout -k 5 60 tools/build/exit_probe init > "$O/init_$k.txt" || exit 1
    e=$(python3 -c 'import time;print("%.6f"%time.monotonic())')
    echo "init probe run $k: $(python3 -c "print('%.1f ms' % (1e3*($e-$s)))")" >> "$O/summary.txt"
  done
fi
for V in ${VARIANTS:-"default:"}; do
  lab=${V%%:*}; envs=${V#*:}; envs=${envs//,/ }
  for k in 1 2 3; do
    sleep 0.5  # as bench.py: a detached worker's driver teardown is not charged to the next run
    env $envs BEDGPU_STATS=1 timeout -k 10 120 python3 tools/e2e_time.py $D/out.bed ./bedops_amd/bin/bedops --intersect $D/A.bed $D/B.bed 2> "$O/${lab}_$k.txt" || { cat "$O/${lab}_$k.txt"; exit 1; }
    echo "$lab $k: $(grep -h '^split' "$O/${lab}_$k.txt") | $(grep -h 'bedgpu host' "$O/${lab}_$k.txt" | awk '{printf "%s%s ", $3, $NF}')" >> "$O/summary.txt"
  done
  sha256sum $D/out.bed | cut -c1-16 >> "$O/summary.txt"
done
cat "$O/summary.txt"
