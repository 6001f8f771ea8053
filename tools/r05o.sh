set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C="timeout -k 10 300 python -u tools/time_convergence.py 4096 3"
for r in 1 2; do
  echo "== round $r tree"; OF2D_CONV_ONLY=1 OF2D_CONV_HASH=1 $C || exit $?
  echo "== round $r gi"; OF2D_CONV_GI=1 OF2D_CONV_ONLY=1 OF2D_CONV_HASH=1 $C || exit $?
  echo "== round $r nt"; OF2D_LIB_PATH=$PWD/tools/abx/nt/libof2d.so OF2D_CONV_ONLY=1 OF2D_CONV_HASH=1 $C || exit $?
  echo "== round $r nt+gi"; OF2D_LIB_PATH=$PWD/tools/abx/nt/libof2d.so OF2D_CONV_GI=1 OF2D_CONV_ONLY=1 OF2D_CONV_HASH=1 $C || exit $?
done > gpurun_out/r05o_gi_nt_ab.log 2>&1
echo rc=$?
