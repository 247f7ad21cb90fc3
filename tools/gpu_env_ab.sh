#!/bin/bash
# env A/B of the intersect bench on one box: the tree as is vs with ENVB set (e.g.
# ENVB="BEDGPU_SET_COLUMNS=1"), REPS alternations, plain and per-kernel (profile-all)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${ROUND:-r06}_${TAG:-envab}; mkdir -p $O
for r in $(seq 1 ${REPS:-2}); do
  for v in a b; do
    for pf in plain prof; do
      A=""; [ $pf = prof ] && A="--profile-all"
      E="$ENVA"; [ $v = b ] && E="$ENVB"
      env $E BG_NOOP=1 timeout -k 10 300 python3 bench.py --workload ${W:-intersect} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-e2e $A > $O/b_${v}_${pf}_$r.json 2> $O/b_${v}_${pf}_$r.err || { tail -5 $O/b_${v}_${pf}_$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/b_${v}_${pf}_$r.json')); print('$v $pf', d['ms_per_step'], d['parity'] and d['parity'].get('matches_reference'), d['roofline']['avg_ms'], d['roofline']['frac']); k=d.get('kernels_ms_per_step'); print(' ', {a: b for a, b in list(k.items())[:12]}) if k else None"
    done
  done
done
