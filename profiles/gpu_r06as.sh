# Round 6, call AS: L7..L1 with 8 waves per workgroup, Lb with 4 (HbCfg): GPU suite, smoke, then ABBA x 2
# against the previous product (4 waves everywhere)
set -e
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06as_gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r06as_gpu_tests.log 2>&1
A=$PWD/deblur-e-nerf_amd/libden_head.so
B=$PWD/deblur-e-nerf_amd/libden.so
bash profiles/ab.sh r06as 1 $A $B
bash profiles/ab.sh r06as 1 $B $A
bash profiles/ab.sh r06as 1 $B $A
bash profiles/ab.sh r06as 1 $A $B
