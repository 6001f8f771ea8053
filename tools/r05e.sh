set -o pipefail
OF2D_LIB_PATH=$PWD/tools/lib_alt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_demons.py > gpurun_out/r05e_divu_tests.log 2>&1 && \
bash tools/gpu_ab_cfg.sh divu 3 3 > gpurun_out/r05e_divu_ab.log 2>&1 && \
bash tools/gpu_ab_conv3.sh 2 cm8 cm16 cm24 cm32 cm16r21 r21s4w3 > gpurun_out/r05e_conv_ab.log 2>&1
echo rc=$?
bash tools/gpu.sh r05e ranksprof
