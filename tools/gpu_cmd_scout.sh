# BEDGPU_SET_SPLIT A/B: the set-load GPU tests (incl. forced splits), then the intersect bench
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05_scout; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_gpu_setload.py tests/test_gpu_parity.py tests/test_gpu_stream.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for s in 1 0 1 0; do
  BEDGPU_SCOUT_SIDE=$s timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/b_$s.json 2> $O/b_$s.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$s.json')); print('scout_side=$s', d['ms_per_step'], d['parity']['matches_reference'], d['roofline']['avg_ms'])"
done
