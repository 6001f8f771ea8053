set -o pipefail
bash tools/gpu.sh r05i tests && \
bash tools/gpu_ab_conv3.sh 2 blk6 blk9 > gpurun_out/r05i_blk_ab.log 2>&1 && \
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05i_bench.log 2>&1
echo rc=$?
