set -o pipefail
bash tools/gpu_ab_conv3.sh 2 pser > gpurun_out/r05h_pser_ab.log 2>&1
bash tools/gpu_ab_chunk.sh 2 12 21 33 > gpurun_out/r05h_chunk_ab.log 2>&1
bash tools/gpu.sh r05h ranksprof
echo rc=$?
