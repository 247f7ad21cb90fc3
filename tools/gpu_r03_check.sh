#!/bin/bash
# Round-3 check on the GPU box: the -m gpu suite, then the headline bench line (e2e + CPU
# baselines), outputs under gpurun_out/r03_<tag>_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-chk}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03_${T}_pytest.log 2>&1 || { tail -30 gpurun_out/r03_${T}_pytest.log; exit 1; }
  tail -3 gpurun_out/r03_${T}_pytest.log
fi
[ -n "$NO_BENCH" ] || timeout -k 10 700 python3 bench.py ${BENCH_ARGS} > gpurun_out/r03_${T}_bench.json 2> gpurun_out/r03_${T}_bench.err || { tail -30 gpurun_out/r03_${T}_bench.err; exit 1; }
cat gpurun_out/r03_${T}_bench.json 2>/dev/null
echo ALLDONE
