# Round 6 (b): the evaluation tests, the in-kernel clock probe (DEN_CLOCK build), the GPU suite,
# smoke(), then a default-length bench line
set -e
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_eval_epoch_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/r06b_eval_tests.log 2>&1
DEN_LIB=deblur-e-nerf_amd/libden_clock.so timeout -k 10 120 python -u profiles/clock_probe.py 3 r06b > gpurun_out/r06b_clock.jsonl 2> gpurun_out/r06b_clock.err
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06b_gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r06b_gpu_tests.log 2>&1
DEN_LIB=deblur-e-nerf_amd/libden_clock.so timeout -k 10 120 python -u profiles/clock_probe.py 3 r06b_after_suite >> gpurun_out/r06b_clock.jsonl 2>> gpurun_out/r06b_clock.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err
echo done
