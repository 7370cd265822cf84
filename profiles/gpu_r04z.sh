# Round 4, call Z: the final tree (every hot kernel page-aligned) as the driver runs it -- GPU suite, smoke,
# the default bench line
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04z_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04z_smoke.log 2>&1
S=$(date +%s)
timeout -k 10 400 python bench.py > gpurun_out/r04z_bench.log 2>&1
echo "bench_wall_s $(( $(date +%s) - S ))" >> gpurun_out/r04z_bench.log
echo done
