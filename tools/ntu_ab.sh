cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_bench.sh r03w_ntu_field 2 - --gpus 1 --steps 10 --warmup 3 --gradients field && bash tools/gpu_ab_bench.sh r03w_ntu_image 2 - --gpus 1 --steps 10 --warmup 3 --gradients image
