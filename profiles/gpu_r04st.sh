set -e
bash profiles/gpu_r04t.sh
bash profiles/gpu_r04s.sh
