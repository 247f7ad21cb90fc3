#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY -- builds the genuine reference tools (BEDOPS v2.4.26) from the
# sources where they lie under /root/reference, into oracle/_ref/ (git-ignored).
#
# This is our own recipe: it does NOT run the reference's system.mk or app Makefiles.
# It compiles, with gcc/g++ directly:
#   - the bundled third-party libraries the reference ships as tarballs
#     (third-party/bzip2-1.0.6, jansson-2.6, zlib-1.2.7), extracted into oracle/_ref/src;
#     jansson's tarball carries its pre-generated src/jansson_config.h, zlib its zconf.h;
#   - interfaces/src/data/{measurement/NaN.cpp, starch/*.c} (compiled as C++, as the
#     reference's app Makefiles do, e.g. applications/bed/bedops/src/Makefile:58-62);
#   - applications/bed/{bedops,bedmap,closestfeats,sort-bed}/src/*.cpp with the
#     reference's own flags (-O3 -std=c++11, static; bedops/src/Makefile:31-32).
# Outputs: oracle/_ref/bin/{bedops,bedmap,closest-features,sort-bed}.
# Used only by tests/golden/make_ref_fixtures.py (fixture generation, here) and by
# bench.py's cpu_baseline leg (the binaries travel to the GPU box; sources do not:
# oracle/_ref/src and oracle/_ref/obj are listed in .gpurunignore).
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$HERE/_ref
if [ ! -d "$REF/applications/bed/bedops/src" ]; then
  echo "build_ref: $REF not present; skipping" >&2
  exit 0
fi
if [ -z "${FORCE:-}" ] && [ -x "$OUT/bin/bedops" ] && [ -x "$OUT/bin/bedmap" ] && \
   [ -x "$OUT/bin/closest-features" ] && [ -x "$OUT/bin/sort-bed" ] && [ "$OUT/bin/bedmap" -nt "$0" ]; then
  exit 0  # already built (FORCE=1 rebuilds)
fi
mkdir -p "$OUT/src" "$OUT/obj" "$OUT/bin"
CC=${CC:-gcc}
CXX=${CXX:-g++}

# 1. third-party sources
for t in bzip2-1.0.6 jansson-2.6 zlib-1.2.7; do
  [ -d "$OUT/src/$t" ] || tar xjf "$REF/third-party/$t.tar.bz2" -C "$OUT/src"
done
BZ=$OUT/src/bzip2-1.0.6
JA=$OUT/src/jansson-2.6/src
ZL=$OUT/src/zlib-1.2.7

build_lib() {  # name cflags sources...
  local name=$1 flags=$2; shift 2
  local objs=()
  mkdir -p "$OUT/obj/$name"
  for s in "$@"; do
    local o="$OUT/obj/$name/$(basename "${s%.*}").o"
    if [ ! -f "$o" ] || [ "$s" -nt "$o" ]; then
      $CC -O2 -w $flags -c "$s" -o "$o" &
    fi
    objs+=("$o")
  done
  wait
  rm -f "$OUT/obj/lib$name.a"
  ar rcs "$OUT/obj/lib$name.a" "${objs[@]}"
}
build_lib bz2 "-D_FILE_OFFSET_BITS=64" \
  $BZ/blocksort.c $BZ/huffman.c $BZ/crctable.c $BZ/randtable.c $BZ/compress.c $BZ/decompress.c $BZ/bzlib.c
# platform feature macros a jansson configure run detects on this Linux/glibc image
JDEF="-DHAVE_STDINT_H=1 -DHAVE_INTTYPES_H=1 -DHAVE_UNISTD_H=1 -DHAVE_SYS_TYPES_H=1 -DHAVE_SYS_STAT_H=1"
JDEF="$JDEF -DHAVE_SYS_TIME_H=1 -DHAVE_SYS_PARAM_H=1 -DHAVE_FCNTL_H=1 -DHAVE_SCHED_H=1 -DHAVE_ENDIAN_H=1"
JDEF="$JDEF -DHAVE_GETPID=1 -DHAVE_GETTIMEOFDAY=1 -DHAVE_OPEN=1 -DHAVE_READ=1 -DHAVE_CLOSE=1"
JDEF="$JDEF -DHAVE_SCHED_YIELD=1 -DHAVE_LOCALECONV=1 -DHAVE_LOCALE_H=1 -DHAVE_SYNC_BUILTINS=1 -DHAVE_ATOMIC_BUILTINS=1 -DUSE_URANDOM=1"
build_lib jansson "-I$JA $JDEF" \
  $JA/dump.c $JA/error.c $JA/hashtable.c $JA/hashtable_seed.c $JA/load.c $JA/memory.c \
  $JA/pack_unpack.c $JA/strbuffer.c $JA/strconv.c $JA/utf.c $JA/value.c
build_lib z "-D_LARGEFILE64_SOURCE=1" \
  $ZL/adler32.c $ZL/compress.c $ZL/crc32.c $ZL/deflate.c $ZL/gzclose.c $ZL/gzlib.c $ZL/gzread.c \
  $ZL/gzwrite.c $ZL/infback.c $ZL/inffast.c $ZL/inflate.c $ZL/inftrees.c $ZL/trees.c $ZL/uncompr.c $ZL/zutil.c

# 2. the reference's interface libraries (NaN + starch), compiled as C++ like its Makefiles
HEAD=$REF/interfaces/general-headers
INC="-iquote$HEAD -I$JA -I$BZ -I$ZL"
FLAGS="-O3 -std=c++11 -w"
mkdir -p "$OUT/obj/iface"
IFACE=()
for s in $REF/interfaces/src/data/measurement/NaN.cpp $REF/interfaces/src/data/starch/*.c; do
  o="$OUT/obj/iface/$(basename "${s%.*}").o"
  [ -f "$o" ] || $CXX -x c++ $FLAGS $INC -c "$s" -o "$o" &
  IFACE+=("$o")
done
wait
LIBS="$OUT/obj/libjansson.a $OUT/obj/libbz2.a $OUT/obj/libz.a"

# 3. the tools
APP=$REF/applications/bed
link() {  # out sources...
  local out=$1; shift
  $CXX -static $FLAGS $INC -o "$OUT/bin/$out" "$@" "${IFACE[@]}" $LIBS
}
link bedops $APP/bedops/src/Bedops.cpp &
link bedmap $APP/bedmap/src/Bedmap.cpp &
link closest-features $APP/closestfeats/src/ClosestFeature.cpp &
link sort-bed $APP/sort-bed/src/Sort.cpp $APP/sort-bed/src/SortDetails.cpp $APP/sort-bed/src/CheckSort.cpp &
wait
for b in bedops bedmap closest-features sort-bed; do
  [ -x "$OUT/bin/$b" ] || { echo "build_ref: $b failed" >&2; exit 1; }
done
echo "build_ref: oracle/_ref/bin/{bedops,bedmap,closest-features,sort-bed} built from $REF"
