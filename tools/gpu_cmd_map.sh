# bedmap A/B (BEDGPU_MAP_BOUNDS): the bedmap GPU tests, then the bedmap bench both ways
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05_${TAG:-map}
mkdir -p $O
timeout -k 10 800 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_bedmap_visitors.py tests/test_gpu_ref_fixtures.py} > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for w in ${WLS:-bedmap}; do
for s in ${SETS:-1 0}; do
  BEDGPU_MAP_BOUNDS=$s timeout -k 10 400 python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --profile-all > $O/$w.$s.json 2> $O/$w.$s.err || { tail -5 $O/$w.$s.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$w.$s.json')); print('$w bounds=$s', d['ms_per_step'], d['parity']['matches_reference'], list(d['kernels_ms_per_step'].items())[:6])"
done
done
