# usage: bash scratch/gpu_ab.sh <tag> <variant>: parity of the variant (render + train tests), then base/variant x2
mkdir -p gpurun_out
export TMPDIR=/tmp
DEN_LIB=$PWD/deblur-e-nerf_amd/libden_$2.so timeout -k 10 400 python -u -m pytest tests/test_render_gpu.py tests/test_train_gpu.py -q --timeout 240 --timeout-method thread > gpurun_out/ab_$1_tests.log 2>&1
echo "variant tests rc=$?"; tail -1 gpurun_out/ab_$1_tests.log
bash profiles/exp_variants.sh $1 base $2 base $2
cat gpurun_out/exp_$1.txt
