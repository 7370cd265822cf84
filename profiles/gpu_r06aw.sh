# Round 6, call AW: Lb's sigma DMA issued by one wave instead of all 8: GPU suite on that build, the
# phase split at 8 waves (all waves recorded), ABBA A/B against the product
set -e
set -o pipefail
mkdir -p gpurun_out
D=$PWD/deblur-e-nerf_amd
DEN_LIB=$D/libden_sig1.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06aw_pytest.log 2>&1
tail -1 gpurun_out/r06aw_pytest.log
DEN_LIB=$D/libden_hidprof.so timeout -k 10 200 python -u profiles/hidden_prof.py 20 > gpurun_out/r06aw_hidden_prof.json 2> gpurun_out/r06aw_hidden_prof.err
A=$D/libden.so; B=$D/libden_sig1.so
bash profiles/ab.sh r06aw 1 $A $B
bash profiles/ab.sh r06aw 1 $B $A
bash profiles/ab.sh r06aw 1 $A $B
bash profiles/ab.sh r06aw 1 $B $A
