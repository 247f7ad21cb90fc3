#!/bin/bash
# quick check: selected GPU tests (TESTS / KEXPR), then the intersect bench (plain and per-kernel)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${ROUND:-r06}_${TAG:-quick}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_T:-600} python -u -m pytest -q -x --timeout 300 --timeout-method thread $TESTS ${KEXPR:+-k "$KEXPR"} > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
  tail -2 $O/pytest.txt
fi
for v in plain prof; do
  A=""; [ $v = prof ] && A="--profile-all"
  timeout -k 10 300 python3 bench.py --workload ${W:-intersect} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-e2e $A > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['ms_per_step'], d['parity'] and d['parity'].get('matches_reference'), d['roofline']['kernel'], d['roofline']['avg_ms'], d['roofline']['frac']); print({k: v for k, v in list((d.get('kernels_ms_per_step') or {}).items())[:14]})"
done
