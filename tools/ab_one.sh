#!/bin/bash
# A/B build of libbedgpu with ONE source recompiled under extra flags, the other objects
# taken from build/obj: tools/ab_one.sh NAME FILE.hip "-DFLAG ..." -> build/ab/NAME/libbedgpu.so
set -e
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
out=build/ab/$name; mkdir -p $out
b=$(basename $src .hip)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-value -Wno-unused-result $* -c $src -o $out/$b.o
objs=$(ls build/obj/*.o | grep -v "/$b.o$")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libbedgpu.so $out/$b.o $objs -L/opt/rocm/lib -lz -ldl -Wl,-rpath,/opt/rocm/lib
echo built $out/libbedgpu.so
