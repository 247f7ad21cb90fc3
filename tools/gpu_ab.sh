#!/bin/bash
# A/B on the GPU box: the -m gpu tests in TESTS under the environment in AB_ENV (e.g.
# BEDGPU_SET_NT=64), then a rocprofv3 kernel table of the bench for each setting in AB_SETS
# ("base" = no extra environment). Outputs under gpurun_out/<ROUND>_<TAG>_*.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-ab}
O=gpurun_out/${ROUND:-r05}_${T}
mkdir -p $O
if [ -n "$TESTS" ]; then
  env $AB_ENV timeout -k 10 ${TEST_TIMEOUT:-900} python3 -u -m pytest $TESTS -m "${MARK:-gpu}" -x -q --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
for S in ${AB_SETS:-base}; do
  E=""
  [ "$S" != "base" ] && E=$(echo "$S" | tr "," " ")
  N=$(echo "$S" | tr '=,' '__')
  env $E timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$N -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e ${BENCH_ARGS} > $O/prof_$N.json 2> $O/prof_$N.err \
    || { tail -20 $O/prof_$N.err; exit 1; }
  f=$(find $O/prof_$N -name '*kernel_stats.csv' | head -1)
  echo "== $S"
  python3 tools/prof_summary.py "$f" $O/kernel_stats_$N.csv || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/prof_$N.json')); print('ms/step', d['ms_per_step'], 'parity', d['parity'])"
done
echo ALLDONE
