#!/bin/bash
# the full GPU test suite with per-test durations, then smoke: gpurun_out/<ROUND>_<TAG>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${ROUND:-r06}_${TAG:-suite}
mkdir -p $O
timeout -k 10 ${SUITE_T:-1000} python -u -m pytest tests -m gpu ${XF--x} -q --timeout 300 --timeout-method thread \
  --durations=${DUR:-60} ${PYTEST_ARGS} > $O/pytest.txt 2>&1
rc=$?
tail -80 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
