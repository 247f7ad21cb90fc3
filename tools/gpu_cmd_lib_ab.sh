# the intersect bench with the in-tree library and with build/ab/<NAMES> (BEDGPU_LIB), alternated
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${ROUND:-r06}_${TAG:-lab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 170 --timeout-method thread -m gpu $TESTS > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for r in $(seq 1 ${REPS:-2}); do
for n in tree ${NAMES}; do
  L=""; [ "$n" != tree ] && L=build/ab/$n/libbedgpu.so
  BEDGPU_LIB=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ${BENCH_ARGS} > $O/b_$n.$r.json 2> $O/b_$n.$r.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$n.$r.json')); print('$n', d['ms_per_step'], d['parity'] and d['parity'].get('matches_reference'), d['roofline']['avg_ms'])"
done
done
