# A/B of build/ab/<NAMES> libraries: loader-stage timing (ab_run.sh style) and the parse
# kernel's FETCH_SIZE / WRITE_SIZE (separate --pmc passes) per variant
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05_abp; mkdir -p $O
for n in ${NAMES:-cur gtxt0}; do
  L=build/ab/$n/libbedgpu.so
  for k in 1 2; do
    BEDGPU_LIB=$L timeout -k 10 200 python3 bench.py --load-only --steps 6 --warmup 1 --no-verify --no-cpu-baseline > $O/t_$n.$k.json 2> $O/t_$n.$k.err || { echo "$n FAILED"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/t_$n.$k.json'));r=d['roofline'];print('%-10s avg %.4f ms step %.3f'%('$n',r['avg_ms'],d['ms_per_step']))"
  done
  BEDGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$n -- python3 bench.py --load-only --steps 1 --warmup 1 --no-verify --no-cpu-baseline > $O/f_$n.json 2> $O/f_$n.err || exit 1
  BEDGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$n -- python3 bench.py --load-only --steps 1 --warmup 1 --no-verify --no-cpu-baseline > $O/w_$n.json 2> $O/w_$n.err || exit 1
  python3 tools/pmc_traffic.py $O/f_$n $O/w_$n $O/pmc_$n.json > /dev/null && python3 -c "
import json; d=json.load(open('$O/pmc_$n.json'))
for k,v in d.items():
  if 'parse' in k: print('$n', k, round(v['bytes']/1e9,3), 'GB/launch read', round(v['read']/1e9,3), 'write', round(v['write']/1e9,3))"
done
