#!/bin/bash
# A/B builds of libbedgpu: tools/ab_build.sh NAME "-DFLAG ..." -> build/ab/NAME/libbedgpu.so
# (run here; the .so files travel with the tree). tools/ab_run.sh times them on the GPU.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=build/ab/$name; mkdir -p $out
objs=()
for f in bedops_amd/csrc/*.hip; do
  o=$out/$(basename $f .hip).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-value -Wno-unused-result $* -c $f -o $o &
  objs+=($o)
done
python3 tools/src_hash.py --flags "ab:$name $*" --write $out/bg_buildhash.c > /dev/null
gcc -O2 -fPIC -c $out/bg_buildhash.c -o $out/bg_buildhash.o
objs+=($out/bg_buildhash.o)
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libbedgpu.so ${objs[@]} -L/opt/rocm/lib -lrccl -lz -ldl -Wl,-rpath,/opt/rocm/lib
echo built $out/libbedgpu.so
