# memory-side atomic requests of the ngp backward (TCC_EA0_ATOMIC) in the configs[3] emulation
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_ATOMIC_sum --output-format csv -d gpurun_out/pmc_atom -o run -- python profiles/bench_ziggy.py --opt-steps 1 --warmup 0 --acc 2 > gpurun_out/pmc_atom.log 2>&1
