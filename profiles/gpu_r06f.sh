# Round 6 (f): the epilogue S' prefetch alone (every build with Lb's dot2 sigma row, so the data are
# identical): none / Lb only / every hidden launch, 4 rounds
set -e
set -o pipefail
export TMPDIR=/tmp
bash profiles/ab.sh r06f 4 deblur-e-nerf_amd/libden_nopf.so deblur-e-nerf_amd/libden_lbpf.so deblur-e-nerf_amd/libden.so
echo done
