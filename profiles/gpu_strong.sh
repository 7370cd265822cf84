# Strong-scaling emulation on one GPU: the per-rank workload of N = 1, 2, 4, 8 ranks (2^17 / N rays),
# bench.py configs[1] otherwise unchanged (no all-reduce: one process).
set -e
mkdir -p gpurun_out
for r in 131072 65536 32768 16384; do
  timeout -k 10 240 python bench.py --rays $r --steps 20 --warmup 3 --no-cpu-baseline --no-gemm-peak --no-extra-legs --psnr-steps 0 > gpurun_out/strong_$r.log 2>&1
done
