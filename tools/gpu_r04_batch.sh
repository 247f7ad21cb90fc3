#!/bin/bash
# Round-4 batch on the GPU box: the -m gpu tests in TESTS, then each step of STEPS:
#   settests    tests/test_gpu_setload.py under BEDGPU_SET_NT=128 (the default is the wave kernel, 64)
#   e2e         bench.py's e2e runs (file, back to back, no detach, pipe)
#   closest_ab  every build/ab/*/libbedgpu.so on the closest 10M x 1B workload (kernel ms)
#   bench:W     rocprof kernel table of bench.py --workload W (W = intersect, bedmap, ...)
#   pmc:W       FETCH_SIZE / WRITE_SIZE passes of bench.py --workload W -> per-kernel traffic json
# Outputs under gpurun_out/r04_<TAG>/. Every GPU step has its own time limit; the script
# stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
T=${TAG:-batch}
O=gpurun_out/r04_${T}
mkdir -p $O
if [ -n "$TESTS" ]; then
  env $TEST_ENV timeout -k 10 ${TEST_TIMEOUT:-900} python3 -u -m pytest $TESTS -m "${MARK:-gpu}" -q --maxfail=${MAXFAIL:-8} --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
for S in $STEPS; do
  case $S in
    settests)  # the set loader's tests under BEDGPU_SET_NT=128 (the round-3 8 KiB-tile kernel)
      BEDGPU_SET_NT=128 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_setload.py -m gpu -x -q --timeout 200 \
        --timeout-method thread > $O/settests.log 2>&1 || { tail -30 $O/settests.log; exit 1; }
      tail -2 $O/settests.log
      ;;
    closest_ab)
      for d in build/ab/*/; do
        n=$(basename $d)
        BEDGPU_LIB=$d/libbedgpu.so timeout -k 10 300 python3 bench.py --workload closest --steps 2 --warmup 1 \
          --no-cpu-baseline --no-e2e > $O/cab_$n.json 2> $O/cab_$n.err || { echo "closest_ab $n FAILED"; tail -5 $O/cab_$n.err; exit 1; }
        python3 -c "import json;d=json.load(open('$O/cab_$n.json'));k=d.get('kernels_first_step_ms',{});print('%-8s step %.1f chunks %s check %s fix %s match %s'%('$n',d['ms_per_step'],k.get('k_closest_chunks'),k.get('k_closest_check'),k.get('k_closest_fix'),d.get('matches_reference')))"
      done
      ;;
    e2e|e2e:*)  # the default workload with its e2e variants (no CPU baseline); e2e:ENV=VAL
      E=""; N=e2e
      case $S in e2e:*) E=${S#e2e:}; N=e2e_$(echo "$E" | tr '=,' '__');; esac
      env $(echo "$E" | tr "," " ") timeout -k 10 600 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/$N.json 2> $O/$N.err || { echo "$N FAILED"; tail -5 $O/$N.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/$N.json'));e=d['e2e'];print('$N', e['median_s'], e['runs_s'], 'b2b', e['back_to_back']['median_s'], 'nodetach', e['no_detach']['median_s'], 'pipe', e['pipe']['median_s'], e['pipe']['runs_s'], 'match', e.get('matches_reference'));print('phases', json.dumps(e.get('phases')))"
      ;;
    closest_cq:*)  # closest_cq:CQ:CW with the main library
      Q=${S#closest_cq:}; CQ=${Q%%:*}; CW=${Q#*:}
      BEDGPU_CLOSEST_CQ=$CQ BEDGPU_CLOSEST_CW=$CW timeout -k 10 300 python3 bench.py --workload closest --steps 2 \
        --warmup 1 --no-cpu-baseline --no-e2e > $O/ccq_${CQ}_$CW.json 2> $O/ccq_${CQ}_$CW.err || { echo "closest_cq $CQ $CW FAILED"; exit 1; }
      python3 -c "import json;d=json.load(open('$O/ccq_${CQ}_$CW.json'));k=d.get('kernels_first_step_ms',{});print('cq %s cw %s step %.1f chunks %s fix %s serial %s'%('$CQ','$CW',d['ms_per_step'],k.get('k_closest_chunks'),k.get('k_closest_fix'),k.get('k_closest_serial')))"
      ;;
    bench:*)  # bench:W or bench:W:ENV=VAL (one extra environment setting)
      W=${S#bench:}
      E=""
      case $W in *:*) E=${W#*:}; W=${W%%:*};; esac
      N=$W$(echo "$E" | tr '=,' '__')
      env $E timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$N -o run -- \
        python3 bench.py --workload $W --steps ${BSTEPS:-5} --warmup 1 --no-cpu-baseline --no-e2e > $O/prof_$N.json \
        2> $O/prof_$N.err || { echo "bench $N FAILED"; tail -20 $O/prof_$N.err; exit 1; }
      f=$(find $O/prof_$N -name '*kernel_stats.csv' | head -1)
      echo "== $N"
      python3 tools/prof_summary.py "$f" $O/kernel_stats_$N.csv || exit 1
      python3 -c "import json; d=json.load(open('$O/prof_$N.json')); print('ms/step', d['ms_per_step'], 'match', (d.get('parity') or {}).get('matches_reference'), 'frac', (d.get('roofline') or {}).get('frac'))"
      ;;
    pmc:*)
      W=${S#pmc:}
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${W}_$C -- python3 bench.py --workload $W \
          --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-verify > $O/pmc_${W}_$C.json 2> $O/pmc_${W}_$C.err \
          || { echo "pmc $W $C FAILED"; tail -5 $O/pmc_${W}_$C.err; exit 1; }
      done
      python3 tools/pmc_traffic.py $O/pmc_${W}_FETCH_SIZE $O/pmc_${W}_WRITE_SIZE $O/pmc_traffic_$W.json || exit 1
      cp $O/pmc_traffic_$W.json profiles/pmc_traffic_$W.json  # read by the bench steps after this one
      echo "pmc $W done"
      ;;
  esac
done
echo ALLDONE
