#!/bin/bash
# row loaders: the GPU tests that read row columns (TESTS), then per workload (WS) the bench
# with the tree's defaults (a: plain + per-kernel) and with ENVB (b: plain)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${ROUND:-r06}_${TAG:-rows}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_T:-700} python -u -m pytest -q -x --timeout 300 --timeout-method thread $TESTS ${KEXPR:+-k "$KEXPR"} > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
  tail -2 $O/pytest.txt
fi
for W in ${WS:-bedmap closest element-of}; do
  for v in a_plain a_prof b_plain; do
    A=""; [ $v = a_prof ] && A="--profile-all"
    E="BG_NOOP=1"; [ ${v%_*} = b ] && E="$ENVB"
    env $E timeout -k 10 400 python3 bench.py --workload $W --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --no-e2e $A > $O/${W}_$v.json 2> $O/${W}_$v.err || { tail -5 $O/${W}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${W}_$v.json')); print('$W $v', d['ms_per_step'], d['parity'] and d['parity'].get('matches_reference'), d['roofline']['kernel'], d['roofline']['avg_ms'], d['roofline']['frac']); k=d.get('kernels_ms_per_step'); print(' ', {a: b for a, b in list(k.items())[:10]}) if k else None"
  done
done
