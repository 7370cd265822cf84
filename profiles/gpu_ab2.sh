# A/B/A/B of libden.so against experiment builds (bench.py configs[1]); usage: bash profiles/gpu_ab2.sh <tag> <v1> [<v2>]
set -e
mkdir -p gpurun_out
tag=$1; shift
bash profiles/exp_variants.sh $tag base "$@" base "$@"
