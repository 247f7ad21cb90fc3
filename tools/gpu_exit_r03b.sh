#!/bin/bash
# process teardown (after-exit) of HIP processes on the box vs what they allocated:
# gpurun_out/exit_r03b/summary.txt (spawner wall clock split by the probe's main/exit stamps)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/exit_r03b; mkdir -p $O
P=./tools/build/exit_probe
run() {  # label runs command...
  local lab=$1 n=$2; shift 2
  for k in $(seq 1 $n); do
    local s=$(python3 -c 'import time;print("%.6f"%time.monotonic())')
    local out
    out=$(timeout -k 5 60 "$@") || { echo "$lab failed" >> $O/summary.txt; return 1; }
    local e=$(python3 -c 'import time;print("%.6f"%time.monotonic())')
    local m=$(echo "$out" | awk '/^main/{print $2}') x=$(echo "$out" | awk '/^exit/{print $2}')
    python3 -c "print('%-14s pre-main %6.1f ms  work %7.1f ms  after-exit %6.1f ms  total %7.1f ms' % ('$lab', 1e3*($m-$s), 1e3*($x-$m), 1e3*($e-$x), 1e3*($e-$s)))" >> $O/summary.txt
  done
}
: > $O/summary.txt
run none 3 $P none
run init 5 $P init
run alloc1 5 $P alloc 1
run alloc16 5 $P alloc 16
run alloc16free 5 $P alloc 16 free
run pin96 5 $P pin 96
run init_full 5 $P init full
cat $O/summary.txt
