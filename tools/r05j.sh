set -o pipefail
bash tools/gpu_ab_conv3.sh 2 pc48 pc80 pc112 > gpurun_out/r05j_pc_ab.log 2>&1
echo rc=$?
