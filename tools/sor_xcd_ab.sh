cd $GRAFT_REPO_ROOT
# The OF2D_SOR_XCD / OF2D_SOR_XCD_LOCALST variants live in commit 06bc2d7 (fluid_kernels.hip);
# not kept: check out that revision to rerun this A/B.
mkdir -p gpurun_out
for r in 1 2; do
for v in base xcd xcdlst; do
  timeout -k 10 60 ./tools/sor_harness_x_$v 8192 8192 4 > gpurun_out/r03q_sor_${v}_8192_$r.log 2>&1 || { echo "$v failed rc=$?"; tail -3 gpurun_out/r03q_sor_${v}_8192_$r.log; exit 1; }
  grep -E "ms \(timeline|hash" gpurun_out/r03q_sor_${v}_8192_$r.log | tail -2 | sed "s/^/$v 8192 r$r: /"
done
done
for v in base xcd xcdlst; do
  timeout -k 10 60 ./tools/sor_harness_x_$v 4096 4096 4 > gpurun_out/r03q_sor_${v}_4096.log 2>&1 || exit 1
  grep -E "ms \(timeline|hash" gpurun_out/r03q_sor_${v}_4096.log | tail -2 | sed "s/^/$v 4096: /"
done
