# parity of the changed kernels, then an A/B/A/B of libden.so against an experiment build
# usage: bash profiles/gpu_ab.sh <tag> <variant>
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_$1.log 2>&1
bash profiles/exp_variants.sh $1 base $2 base $2
