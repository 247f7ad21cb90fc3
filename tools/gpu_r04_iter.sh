#!/bin/bash
# Round-4 iteration on the GPU box: selected -m gpu tests (TESTS, default: the whole suite),
# then a kernel table of the bench under rocprofv3 (BENCH_ARGS), then optionally the plain
# bench line (FULL_BENCH=1). Outputs under gpurun_out/r04_<TAG>_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-it}
O=gpurun_out/r04_${T}
mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python3 -u -m pytest ${TESTS:-tests} -m "${MARK:-gpu}" -x -q --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
if [ -z "$NO_PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e ${BENCH_ARGS} > $O/prof_bench.json 2> $O/prof_bench.err \
    || { tail -20 $O/prof_bench.err; exit 1; }
  f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
  python3 tools/prof_summary.py "$f" $O/kernel_stats.csv || exit 1
  cat $O/prof_bench.json
fi
if [ -n "$FULL_BENCH" ]; then
  timeout -k 10 700 python3 bench.py ${FULL_ARGS} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
echo ALLDONE
