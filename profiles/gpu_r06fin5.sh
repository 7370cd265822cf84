# Round 6 final tree (pe weight gradients folded into L5 / L1; every hidden launch at 8 waves; bench defaults W = 10, K = 20): kernel trace +
# FETCH / WRITE PMC + two SQ passes, GPU suite, smoke, default bench
set -e
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
P="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0"
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06fin5_prof -o run -- $B > gpurun_out/r06fin5_prof.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r06fin5_pmc_fetch -o run -- $P > gpurun_out/r06fin5_pmc_fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r06fin5_pmc_write -o run -- $P > gpurun_out/r06fin5_pmc_write.log 2>&1
PMC1=$(python profiles/pick_counters.py gpurun_out/counters.txt SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE)
echo "pass1: $PMC1" > gpurun_out/r06fin5_pmc_sets.txt
timeout -s KILL 150 rocprofv3 --pmc $PMC1 --output-format csv -d gpurun_out/r06fin5_pmc_mfma -o run -- $P > gpurun_out/r06fin5_pmc_mfma.log 2>&1
PMC2=$(python profiles/pick_counters.py gpurun_out/counters.txt SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE)
echo "pass2: $PMC2" >> gpurun_out/r06fin5_pmc_sets.txt
timeout -s KILL 150 rocprofv3 --pmc $PMC2 --output-format csv -d gpurun_out/r06fin5_pmc_mfma2 -o run -- $P > gpurun_out/r06fin5_pmc_mfma2.log 2>&1
rm -f gpurun_out/r06fin5_prof/run_agent_info.csv
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r06fin5_gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r06fin5_gpu_tests.log 2>&1
timeout -k 10 500 python -u bench.py > gpurun_out/r06fin5_bench_default.json 2> gpurun_out/r06fin5_bench.err
echo done
