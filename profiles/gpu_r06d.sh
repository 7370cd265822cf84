# Round 6 (d): Lb's sigma weight-gradient row by VALU dot products instead of a dependent MFMA chain:
# the gradient tests first, the phase split of the new build, then a same-box A/B against HEAD's build
set -e
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_render_gpu.py tests/test_deblur_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r06d_tests.log 2>&1
DEN_LIB=deblur-e-nerf_amd/libden_hidprof.so timeout -k 10 180 python -u profiles/hidden_prof.py 20 > gpurun_out/r06d_hidden_prof.json 2> gpurun_out/r06d_hidden_prof.err
bash profiles/ab.sh r06d 3 deblur-e-nerf_amd/libden_base.so deblur-e-nerf_amd/libden.so
echo done
