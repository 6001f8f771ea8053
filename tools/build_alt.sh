#!/bin/bash
# Build tools/lib_alt.so: the in-tree objects with the listed sources taken
# from git revision <rev> (the B side of tools/gpu_ab_bench.sh).
#   tools/build_alt.sh <rev> <source under opticalflow2d_amd/csrc>...
set -e
cd "$(dirname "$0")/.."
C=opticalflow2d_amd/csrc
rev=$1; shift
make -C $C -j8 > /dev/null
D=$(mktemp -d)
trap 'rm -rf $D' EXIT
T=$D/src/csrc  # ../../include/of2d.h resolves to $D/include
mkdir -p $T $D/include
cp include/of2d.h $D/include/
cp $C/*.h $C/*.hip $C/*.cpp $T/
for f in "$@"; do git show "$rev:$C/$f" > "$T/$f"; done
# a replaced header: every object is rebuilt (class layouts must agree)
allh=0
for f in "$@"; do case $f in *.h) allh=1;; esac; done
objs=""
for o in $C/build/*.o; do
  b=$(basename "$o" .o); src=""
  for f in "$@"; do [ "${f%.*}" = "$b" ] && src=$f; done
  if [ $allh = 1 ] && [ -z "$src" ]; then
    for e in hip cpp; do [ -f "$T/$b.$e" ] && src=$b.$e; done
  fi
  if [ -n "$src" ]; then
    /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-pass-failed --offload-arch=gfx950 \
      -I/opt/rocm/include -munsafe-fp-atomics -x hip -c "$T/$src" -o "$T/$b.o"
    objs="$objs $T/$b.o"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o tools/lib_alt.so $objs
echo "tools/lib_alt.so: $* at $rev"
