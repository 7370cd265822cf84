# Round 6, call N: dz_l written over S_{l+1} instead of S_l (stream probe: 5.50 -> 5.81 TB/s for the pattern).
# GPU suite on the new build, then A/B against the previous build (libden_base.so), 3 alternating rounds.
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06n_gpu_tests.log 2>&1
bash profiles/ab.sh r06n 3 $PWD/deblur-e-nerf_amd/libden_base.so $PWD/deblur-e-nerf_amd/libden.so
