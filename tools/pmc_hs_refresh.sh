cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I opticalflow2d_amd/csrc tools/hs_variants.hip -o tools/hs_variants > gpurun_out/r03bv_build.log 2>&1 || exit 1
bash tools/gpu_pmc_bench.sh && cp gpurun_out/pmcb/hs_traffic.json gpurun_out/r03bv_hs_traffic.json && cat gpurun_out/r03bv_hs_traffic.json | head -30
