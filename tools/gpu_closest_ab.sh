cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k closest -x -q --timeout 200 --timeout-method thread > gpurun_out/cl_tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cl_trace -- python3 bench.py --workload closest --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/cl_trace.json 2> gpurun_out/cl_trace.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/cl_fetch -- python3 bench.py --workload closest --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-verify > gpurun_out/cl_fetch.json 2> gpurun_out/cl_fetch.err || exit 1
echo done
