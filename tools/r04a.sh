set -o pipefail
bash tools/gpu_ranks.sh && bash tools/grid_write_probe.sh "1 2 4 8"
