#!/bin/bash
# Stage ablation of the Demons fused kernel (OF2D_DEMONS_ABL, timing only).
#   build (here):  tools/demons_abl.sh build
#   run (GPU box): tools/demons_abl.sh run <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
C=opticalflow2d_amd/csrc
if [ "$1" = build ]; then
  mkdir -p $C/build_abl
  for n in 0 1 2 3 4; do
    /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-pass-failed --offload-arch=gfx950 \
      -munsafe-fp-atomics -DOF2D_DEMONS_ABL=$n -x hip -c $C/demons_kernels.hip -o $C/build_abl/demons_$n.o || exit 1
    objs=$(ls $C/build/*.o | grep -v demons_kernels.o)
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib \
      -o tools/lib_abl_$n.so $objs $C/build_abl/demons_$n.o || exit 1
  done
  exit 0
fi
tag=$2
export TMPDIR=/tmp
mkdir -p gpurun_out/$tag
for n in 0 1 2 3 4; do
  OF2D_LIB_PATH=$PWD/tools/lib_abl_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $PWD/gpurun_out/$tag/abl$n -o k -- python3 $PWD/bench_configs.py --configs 3 > gpurun_out/$tag/abl$n.log 2>&1 || exit $?
  python3 - "$PWD/gpurun_out/$tag/abl$n/k_kernel_stats.csv" $n <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'demons_fused' in r['Name'] or 'smooth_norm' in r['Name']:
        print('abl', sys.argv[2], r['Name'][:48], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
