# round-5 A/B: tests touched by the side-stream set merge, the equal-row ranking and the
# wave closest kernel; then intersect (BEDGPU_SET_SIDE) and closest (BEDGPU_CLOSEST_WAVE) benches
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05_${TAG:-side}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_bedmap_visitors.py tests/test_gpu_ref_fixtures.py tests/test_gpu_setload.py tests/test_gpu_parity.py} > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for s in ${SIDE_SETS-1 0 1 0}; do
  BEDGPU_SET_SIDE=$s timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/b_$s.json 2> $O/b_$s.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$s.json')); print('side=$s', d['ms_per_step'], d['parity'], d['roofline']['avg_ms'])"
done
for w in ${CL_SETS-BEDGPU_CLOSEST_WAVE=1 BEDGPU_CLOSEST_WAVE=0}; do
  N=$(echo "$w" | tr '=,' '__')
  env $(echo "$w" | tr ',' ' ') timeout -k 10 400 python3 bench.py --workload closest --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --profile-all > $O/c_$N.json 2> $O/c_$N.err || exit 1
  python3 -c "import json; d=json.load(open('$O/c_$N.json')); print('$w', d['ms_per_step'], d['parity'], list(d['kernels_ms_per_step'].items())[:4])"
done
