set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_workloads.py > gpurun_out/r05d_workloads.log 2>&1; echo "workloads rc=$?"
bash tools/gpu_ab_conv3.sh 2 cm16 cm16c cm32c r21s4w3 r27s4w4 > gpurun_out/r05d_conv_ab.log 2>&1 && \
bash tools/gpu.sh r05d ranksprof
echo rc=$?
