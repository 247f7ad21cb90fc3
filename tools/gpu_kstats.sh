#!/bin/bash
# kernel table of the headline bench (or BENCH_ARGS) under rocprofv3; gpurun_out/ks_<TAG>/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ks_${TAG:-x}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
r = list(csv.reader(open(sys.argv[1])))
for x in r[1:20]:
    print("%-44s %5s %9.1f us" % (x[0][:44], x[1], float(x[3]) / 1e3))
PY
