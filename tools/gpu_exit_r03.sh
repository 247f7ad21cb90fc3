#!/bin/bash
# process start/exit costs of HIP processes on the box: outputs gpurun_out/exit_r03/*.txt
# (each line: the mode, the spawner's wall clock, and the probe's main/exit stamps)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/exit_r03; mkdir -p $O
D=/tmp/e2e; mkdir -p $D
[ -f $D/A.bed ] || ./tools/build/bedgen 100000000 42 > $D/A.bed || exit 1
P=./tools/build/exit_probe
run() {  # label command...
  local lab=$1; shift
  for k in 1 2 3; do
    local s=$(python3 -c 'import time;print("%.6f"%time.monotonic())')
    local out
    out=$(timeout -k 5 60 "$@") || { echo "$lab failed" >> $O/summary.txt; return 1; }
    local e=$(python3 -c 'import time;print("%.6f"%time.monotonic())')
    local m=$(echo "$out" | awk '/^main/{print $2}') x=$(echo "$out" | awk '/^exit/{print $2}')
    python3 -c "print('%-22s pre-main %6.1f ms  work %7.1f ms  after-exit %6.1f ms  total %7.1f ms' % ('$lab', 1e3*($m-$s), 1e3*($x-$m), 1e3*($e-$x), 1e3*($e-$s)))" >> $O/summary.txt
    echo "$out" > $O/${lab}_$k.txt
  done
}
: > $O/summary.txt
run s0 $P streams 0
run s1 $P streams 1
run s3 $P streams 3
run s8 $P streams 8
run s0_q1 env GPU_MAX_HW_QUEUES=1 $P streams 0
run s3_q1 env GPU_MAX_HW_QUEUES=1 $P streams 3
run s3_q2 env GPU_MAX_HW_QUEUES=2 $P streams 3
run s1_vis env HIP_VISIBLE_DEVICES=0 $P streams 1
for f in $O/s*_1.txt; do echo "$f: $(grep setdevice $f)" >> $O/summary.txt; done
cat $O/summary.txt
