#!/bin/bash
# one pytest selection under rocprofv3 kernel stats; outputs gpurun_out/tp_<TAG>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/tp_${TAG:-x}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && head -15 "$f" | cut -d, -f1-4
exit $rc
