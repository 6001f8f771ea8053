set -o pipefail
bash tools/gpu.sh r05b sntests && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hs.py > gpurun_out/r05b_hstests.log 2>&1 && \
OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 3 > gpurun_out/r05b_conv.log 2>&1 && \
bash tools/gpu_sor_abl.sh 2 8192 8192 0 1 2 4 8 16 6 7 15 > gpurun_out/r05b_sor_abl.log 2>&1 && \
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05b_bench.log 2>&1
echo rc=$?
