#!/bin/bash
# Build libof2d.so with extra compile flags for one source into tools/abx/<name>/ (travels to the GPU box; tools/ab/ does not)
# (an A/B variant; the in-tree objects for everything else):
#   [REV=<git rev>] tools/build_variant.sh <name> <source under csrc> <flags...>
# (REV: that revision's text of the source, compiled beside today's headers)
set -e
cd "$(dirname "$0")/.."
C=opticalflow2d_amd/csrc
name=$1 src=$2; shift 2
make -C $C -j8 > /dev/null
D=tools/abx/$name
mkdir -p $D
b=$(basename "$src" .hip); b=$(basename "$b" .cpp)
SRC=$C/$src
if [ -n "$REV" ]; then
    SRC=$C/.variant_$b.${src##*.}
    git show "$REV:$C/$src" > $SRC
    trap 'rm -f $SRC' EXIT
fi
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-pass-failed --offload-arch=gfx950 \
    -I/opt/rocm/include -munsafe-fp-atomics "$@" -x hip -c $SRC -o $D/$b.o
objs=""
for o in $C/build/*.o; do
    if [ "$(basename "$o" .o)" = "$b" ]; then objs="$objs $D/$b.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o $D/libof2d.so $objs
rm -f $D/$b.o
echo "$D/libof2d.so: $src $*"
