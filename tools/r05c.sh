set -o pipefail
bash tools/gpu.sh r05c sntests && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hs.py > gpurun_out/r05c_hstests.log 2>&1 && \
OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 3 > gpurun_out/r05c_conv.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05c_convprof -o k -- python3 -u tools/time_convergence.py 4096 1 > gpurun_out/r05c_convprof.log 2>&1 && \
bash tools/gpu_sor_abl.sh 2 8192 8192 0 36 38 39 63 > gpurun_out/r05c_sor_abl.log 2>&1
echo rc=$?
