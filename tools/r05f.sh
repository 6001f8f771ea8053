set -o pipefail
bash tools/gpu.sh r05f sntests && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hs.py tests/test_gpu_ranks.py > gpurun_out/r05f_hsranks.log 2>&1 && \
OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 3 > gpurun_out/r05f_conv.log 2>&1 && \
bash tools/gpu.sh r05f texprof
echo rc=$?
bash tools/gpu.sh r05f ranksprof
