export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05_side
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bedmap_visitors.py tests/test_gpu_ref_fixtures.py tests/test_gpu_setload.py > gpurun_out/r05_side/pytest.log 2>&1 || { tail -30 gpurun_out/r05_side/pytest.log; exit 1; }
tail -2 gpurun_out/r05_side/pytest.log
for s in 1 0 1 0; do
  BEDGPU_SET_SIDE=$s timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r05_side/b_$s.json 2> gpurun_out/r05_side/b_$s.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r05_side/b_$s.json')); print('side=$s', d['ms_per_step'], d['parity'], d['roofline']['avg_ms'])"
done
