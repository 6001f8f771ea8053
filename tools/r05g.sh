set -o pipefail
bash tools/gpu.sh r05g slabtests ranks
echo rc=$?
