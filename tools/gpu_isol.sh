# the failing sharded bedmap case outside pytest, HIP's API log (AMD_LOG_LEVEL=3) of the failing run
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/isol
AMD_LOG_LEVEL=3 timeout -k 10 200 python3 tools/isol_shard.py; echo rc=$?
grep -n "Invalid\|invalid\|Error\|error" gpurun_out/isol/stderr.txt | head -20
