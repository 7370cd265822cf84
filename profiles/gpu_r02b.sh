# Round 2, call B: the new parity tests (packed rendering, trajectory, DeblurENeRF.training_step),
# then the whole GPU suite.  A test failure (pytest rc 1) does not stop the script; anything else
# (fault, abort, timeout) does.
mkdir -p gpurun_out
export TMPDIR=/tmp
rc=0
timeout -k 10 600 python -u -m pytest tests/test_nerfacc_gpu.py tests/test_deblur_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/t_new.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
rc=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --ignore=tests/test_nerfacc_gpu.py --ignore=tests/test_deblur_gpu.py > gpurun_out/t_all.log 2>&1 || rc=$?
exit $rc
