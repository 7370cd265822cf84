# Round 6, call P: S_0..S_7 / dz_0..dz_7 as block-major 144 KiB rows (stream probe: 6.23 TB/s for a hidden
# launch's pattern within one row).  GPU suite on the new build, then A/B against the r06n build.
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06p_gpu_tests.log 2>&1
bash profiles/ab.sh r06p 3 $PWD/deblur-e-nerf_amd/libden_r06n.so $PWD/deblur-e-nerf_amd/libden.so
