# BEDGPU_MAP_STAGE A/B: bedmap GPU tests (visitors + bedmap fixtures), then the bedmap bench both ways
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05_map2; mkdir -p $O
BEDGPU_MAP_STAGE=1 timeout -k 10 800 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu tests/test_gpu_bedmap_visitors.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for s in 1 0 1 0; do  # (1: staged ends and scores)
  BEDGPU_MAP_STAGE=$s timeout -k 10 400 python3 bench.py --workload bedmap --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --profile-all > $O/b_$s.json 2> $O/b_$s.err || { tail -5 $O/b_$s.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$s.json')); print('stage=$s', d['ms_per_step'], d['parity']['matches_reference'], d['kernels_ms_per_step'].get('k_map_ops'))"
done
