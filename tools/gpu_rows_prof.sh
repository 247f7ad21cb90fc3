#!/bin/bash
# per-launch kernel times of one workload under rocprofv3 --kernel-trace, the tree's defaults
# (a) against ENVB (b): gpurun_out/<ROUND>_<TAG>/<W>_{a,b}/...kernel_trace.csv + a summary
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${ROUND:-r06}_${TAG:-rprof}; mkdir -p $O
for W in ${WS:-bedmap}; do
  for v in a b; do
    E="BG_NOOP=1"; [ $v = b ] && E="$ENVB"
    export $E
    timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/${W}_$v -o run -- python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/${W}_$v.json 2> $O/${W}_$v.err || { tail -5 $O/${W}_$v.err; exit 1; }
    unset ${E%%=*}
    python3 - "$O/${W}_$v" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    d[r["Kernel_Name"][:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print(sys.argv[1].split("/")[-1], k, len(v), [round(x) for x in v[-6:]])
PY
  done
done
