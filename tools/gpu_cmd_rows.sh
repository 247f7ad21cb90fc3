# scout-free row loads (k_parse_n look-back): the row-loader GPU tests, then bedmap / closest /
# element-of benches with and without the scout pass (BEDGPU_ROW_SCOUT=1)
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05_${TAG:-rows}
mkdir -p $O
if [ -n "${TESTS-x}" ]; then
timeout -k 10 800 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_setload.py tests/test_gpu_parity.py tests/test_gpu_ref_fixtures.py tests/test_gpu_stream.py} > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
fi
for w in ${WLS:-bedmap closest element-of}; do
for s in ${SCOUT_SETS:-0 1}; do
  BEDGPU_ROW_SCOUT=$s timeout -k 10 400 python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --profile-all > $O/$w.$s.json 2> $O/$w.$s.err || { tail -5 $O/$w.$s.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.$s.json')); print('$w scout=$s', d['ms_per_step'], d['parity']['matches_reference'], list(d['kernels_ms_per_step'].items())[:5])"
done
done
