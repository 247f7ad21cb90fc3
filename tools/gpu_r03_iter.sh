#!/bin/bash
# round-3 iteration on the GPU box: selected GPU tests, device-step A/B of bench.py under env
# variants, e2e variants of the CLI. Env: TESTS (pytest args), BENCH_VARIANTS ("label:ENV=V,.."),
# E2E_VARIANTS (as tools/gpu_e2e_var.sh), TAG. Outputs under gpurun_out/iter_<TAG>/.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/iter_${TAG:-x}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit 1
fi
for V in $BENCH_VARIANTS; do
  lab=${V%%:*}; envs=${V#*:}; envs=${envs//,/ }
  env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e ${BENCH_ARGS} > $O/bench_$lab.json 2> $O/bench_$lab.err || { tail -20 $O/bench_$lab.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$lab.json'));r=d['roofline'];print('$lab', d['ms_per_step'], 'ms/step', r['kernel'], r['avg_ms'], 'ms frac', r['frac'])"
done
if [ -n "$E2E_VARIANTS" ]; then TAG=${TAG:-x} VARIANTS="$E2E_VARIANTS" tools/gpu_e2e_var.sh || exit 1; fi
echo ALLDONE
