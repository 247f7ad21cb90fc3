# one full bench.py line for a workload (device step, e2e file->file with its variants, the
# reference's --chrom fan-out on the box's CPUs, run (i) from the pin file), plus its
# rocprofv3 kernel table: gpurun_out/<ROUND>_cfg_<W>.{json,err}, ..._kernel_stats.csv
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
W=${WORKLOAD:-bedmap}
O=gpurun_out/${ROUND:-r05}_cfg_$W
mkdir -p $O
df -h /tmp > $O/df.txt 2>&1; nproc >> $O/df.txt
timeout -k 10 ${BENCH_T:-1000} python3 bench.py --workload $W --steps ${STEPS:-5} --warmup 1 --cpu-single-runs 0 \
  --cpu-fanout-runs ${FAN_RUNS:-3} ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d['parity'], d.get('e2e_intervals_per_s'), d.get('gpu_vs_cpu'), (d.get('e2e') or {}).get('matches_reference'))"
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --workload $W --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
  f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
  python3 tools/prof_summary.py "$f" $O/kernel_stats.csv | head -12
fi
